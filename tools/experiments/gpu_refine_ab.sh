# k_refine_exact / k_refine_fast durations and counts, default library vs variants (isolated detections)
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for v in default "$@"; do
  L=""; [ $v != default ] && L=$R/build_var/$v.so
  ( cd /tmp; SIFT_HIP_LIB=$L SIFT_DEBUG_REFINE=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/rab_$v -o run -- python $R/tools/refine_bounds.py > $R/gpurun_out/rab_$v.log 2>&1 ) || { echo "$v failed"; tail -5 $R/gpurun_out/rab_$v.log; exit 1; }
  echo "== $v"; grep -E "^3840|refine uncertain" $R/gpurun_out/rab_$v.log | head -3
  python3 - $R/gpurun_out/rab_$v/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Kernel_Name"]
    if "refine" in n:
        print("  ", n[:28], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
done
