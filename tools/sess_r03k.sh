# round-3 session: rocprofv3 kernel trace + FETCH/WRITE of the complex128 configs, a 2-rank
# rehearsal of bench.py --gpus 2 (gloo, both ranks on the one GPU), 4-wave complex128 RX A/B
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in b c d e; do
  PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03k_${c}_f64 --config $c --precision f64 > gpurun_out/r03k_prof_$c.txt 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/r03k_prof_$c.txt; exit 1; }
  echo "profile $c ok"
done
OFDM_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 --symbols 200000 --no-cpu-baseline --no-ber-check > gpurun_out/r03k_bench_2rank.json 2> gpurun_out/r03k_bench_2rank.err; rc=$?
echo "2-rank rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03k_bench_2rank.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/r03k_bench_2rank.json')); print(d['n_gpus'], d['devices'], '%.4g'%d['value'], d['dtype'])"
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base rx1024" "b" 2>&1 | grep -v amdgpu.ids
