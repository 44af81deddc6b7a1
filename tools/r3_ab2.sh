# GPU parity suite on this build, then a same-box A/B vs the session-start build in three regimes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3g_gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_modes.sh 2 main r3base > gpurun_out/r3g_ab_modes.txt 2>&1 || exit 1
