#!/bin/bash
# round-6 final-tree session: GPU suite, bench, rocprof kernel stats, single-pass and shard rehearsals
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06z}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench rc=$?; tail $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 240 python tools/single_pass.py --passes 20 > $OUT/single.txt 2>&1 || { echo single failed; exit 1; }
timeout -k 10 240 python tools/shard_rehearsal.py --sync --steps 10 > $OUT/rehearsal_sync.txt 2>&1 || { echo reh-sync failed; exit 1; }
timeout -k 10 240 python tools/shard_rehearsal.py --steps 20 > $OUT/rehearsal.txt 2>&1 || { echo reh failed; exit 1; }
grep -v '^{' $OUT/single.txt; grep -v '^{' $OUT/rehearsal_sync.txt; grep -v '^{' $OUT/rehearsal.txt
exit 0
