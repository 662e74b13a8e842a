#!/bin/bash
# Copy the round artifacts of tools/gpu_round.sh <tag> from gpurun_out/ into profiles/.
# usage: tools/save_profiles.sh <tag>
set -e
T=$1
R=$(cd "$(dirname "$0")/.." && pwd)
G=$R/gpurun_out
P=$R/profiles
python3 $R/tools/pmc_launches.py --config-key 3840x2160_o4_s5 --round $T --out $P/${T}_pmc_4k_o4_s5.json $G/pmc_${T}_FETCH_SIZE $G/pmc_${T}_WRITE_SIZE $G/pmc_${T}_TA $( [ -d $G/pmc_${T}_SQ ] && echo $G/pmc_${T}_SQ ) > $P/${T}_pmc_4k_o4_s5.txt
cp $G/prof_${T}/run_kernel_stats.csv $P/${T}_4k_o4_s5_kernel_stats.csv
cp $G/prof_${T}_iso/run_kernel_stats.csv $P/${T}_iso_4k_o4_s5_kernel_stats.csv
python3 $R/tools/kstats.py $P/${T}_4k_o4_s5_kernel_stats.csv > $P/${T}_4k_o4_s5_kernel_stats.txt
python3 $R/tools/kstats.py $P/${T}_iso_4k_o4_s5_kernel_stats.csv > $P/${T}_iso_4k_o4_s5_kernel_stats.txt
cp $G/bench_${T}.json $P/${T}_bench.json
cp $G/bench_prof_${T}.json $P/${T}_bench_under_rocprof.json
cp $G/bench_prof_${T}_iso.json $P/${T}_iso_bench_under_rocprof.json
python3 $R/tools/gauss_oct.py $G/prof_${T}_iso/run_kernel_trace.csv $G/prof_${T}/run_kernel_trace.csv > $P/${T}_per_octave_trace.txt
[ -f $G/pytest_gpu_${T}.log ] && cp $G/pytest_gpu_${T}.log $P/${T}_pytest_gpu.log
cp $G/smoke_${T}.log $P/${T}_smoke.log
echo saved $T
