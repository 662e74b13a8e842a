#!/bin/bash
# On the GPU box: one bench step with the refinement diagnostics printed.
cd ${GRAFT_REPO_ROOT:-$(pwd)} && SIFT_DEBUG_REFINE=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline 2>&1 | tail -4 | cut -c1-300
