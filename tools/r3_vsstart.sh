# same-box A/B of the shipped engine vs the round-3 session-start engine (c952bab) in three regimes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/ab_modes.sh 2 main r3start > gpurun_out/r3t_ab_vs_start.txt 2>&1 || exit 1
