#!/bin/bash
# tests/example/run_example.sh with the MI355X drop-in pieces (run from a copy
# of tests/golden/example): PIPSORT, then global and not-shared PIPs.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
"$ROOT/pipsort_amd/bin/PIPSORT" -c 2 -l ldfiles.txt -z zfiles.txt -m snp_map -n 334324,6771 -p 0.25 -o pipsort_results
PYTHONPATH="$ROOT" python -m pipsort_amd.postprocess global pipsort_results_study0_post.txt pipsort_results_study1_post.txt pipsort_results_shared_pips.txt global_pips.txt
PYTHONPATH="$ROOT" python -m pipsort_amd.postprocess notshared pipsort_results_shared_pips.txt global_pips.txt not_shared_pips.txt
