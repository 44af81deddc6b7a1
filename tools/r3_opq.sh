# same-box A/B: throughput launches on the ahead-of-time kernel vs the compiled configuration with opaque
# replica-layout offsets (variant library "opq")
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/ab_mix.sh 3 multi aot:main:base opq_jit:opq:PRIMEUNCORE_JIT_THROUGHPUT=1 > gpurun_out/r3o_ab_opq.txt 2>&1 || exit 1
