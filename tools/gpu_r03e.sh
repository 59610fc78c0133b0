export TMPDIR=/tmp
OUT=gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh 1,8 3 - _ab/base || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/cfg -o run -- python3 tools/configs_time.py > $OUT/cfg.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sss -o run -- python3 tools/sss_time.py --M 200 --c 5 --reps 2 > $OUT/sss.log 2>&1 || exit $?
