# wide-set goldens + JIT tests, same-box A/B of this build vs the session-start build (r3base), then profiles
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -k "128way or 192way or jit or ahead" > gpurun_out/r3b_wide_tests.log 2>&1 || exit 1
timeout -k 10 500 bash tools/ab_multi.sh 2 main r3base > gpurun_out/r3b_ab_multi.txt 2>&1 || exit 1
AB_OTHER=r3base timeout -k 10 300 bash tools/ab_single.sh > gpurun_out/r3b_ab_single.txt 2>&1 || exit 1
bash tools/r3_prof.sh r3b
