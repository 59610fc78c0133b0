mkdir -p gpurun_out/r03w
for L in "" $PWD/_ab/abl1/libpipsort_engine.so; do
  n=$(basename $(dirname ${L:-x/base/y}))
  PSX_ENGINE_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03w/$n -o run -- python3 tools/sss_time.py --M 200 --c 5 --reps 2 > gpurun_out/r03w/$n.log 2>&1 || exit 1
done
