# round-3 session: complex128 ablation timings (diagnostic build) of configs c and e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/ablate.py --config c --precision f64 --symbols 1000000 > gpurun_out/r03t_ablate_c.txt 2>&1 || { tail -5 gpurun_out/r03t_ablate_c.txt; exit 1; }
timeout -k 10 300 python -u tools/ablate.py --config e --precision f64 --symbols 250000 > gpurun_out/r03t_ablate_e.txt 2>&1 || { tail -5 gpurun_out/r03t_ablate_e.txt; exit 1; }
timeout -k 10 300 python -u tools/ablate.py --config b --precision f64 --symbols 1000000 > gpurun_out/r03t_ablate_b.txt 2>&1 || { tail -5 gpurun_out/r03t_ablate_b.txt; exit 1; }
grep -v '^{' gpurun_out/r03t_ablate_c.txt gpurun_out/r03t_ablate_e.txt gpurun_out/r03t_ablate_b.txt
