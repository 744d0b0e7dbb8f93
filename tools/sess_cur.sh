set -o pipefail
TAG=r04b NO_BENCH=1 tools/gpu_session.sh || exit $?
AB_REPS=2 AB_STEPS=30 timeout -k 10 600 bash tools/ab.sh "old default h3" "c d e" 2>&1 | tee gpurun_out/r04b_ab.txt
