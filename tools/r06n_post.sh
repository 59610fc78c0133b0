for m in 0 1 0 1; do
  if [ $m = 1 ]; then export PSX_BENCH_STEPSYNC=1; else unset PSX_BENCH_STEPSYNC; fi
  echo "== PSX_BENCH_STEPSYNC=$m"
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('single_pass_ms'), d.get('pass_mode'))" || exit 1
done
