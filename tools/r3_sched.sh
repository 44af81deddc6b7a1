# same-box A/B: the throughput launches on the ahead-of-time kernel vs the compiled configuration under
# three machine-scheduler strategies (jit.cpp options)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_mix.sh 2 multi aot:main:base jit_ilp:main:PRIMEUNCORE_JIT_THROUGHPUT=1 jit_occ:jocc:PRIMEUNCORE_JIT_THROUGHPUT=1 jit_mem:jmem:PRIMEUNCORE_JIT_THROUGHPUT=1 > gpurun_out/r3m_ab_sched.txt 2>&1 || exit 1
