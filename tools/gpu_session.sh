#!/bin/bash
# One GPU-box session: run the named steps in order, each under its own time
# limit, stopping at the first failure (no step is retried).  Outputs go to
# gpurun_out/TAG_*.  Replaces round 3's one-off tools/r3_*.sh scripts.
#
#   tools/gpu_session.sh TAG STEP [STEP ...]
#
# Steps:
#   tests        pytest -m gpu (the whole GPU parity suite)
#   smoke        __graft_entry__.smoke()
#   latency      tools/latency_bench.py: uncore_access and one message per call, resident kernel vs a launch per call
#   traffic      PMC fabric traffic of the headline kernel on the driver's window (tools/pmc_traffic.py)
#   bench        bench.py on the driver's config (--steps 20 --warmup 5), carrying TAG_traffic.json if present
#   bench_default  bench.py with no flags
#   bench_c3 / bench_c5  bench.py --config C3 / C5 on the driver's window (C5 closed loop by default)
#   rocprof      rocprofv3 --kernel-trace --stats of the driver's config (headline only)
#   sq           SQ wave-state / instruction counters of the headline kernel (tools/pmc_sq.py)
#   sq_closed / traffic_closed / regions_closed  the headline kernel's SQ counters, fabric traffic and region
#                profile on the closed-loop replay of the same workload (bench --replay closed)
#   sq_single    the same for one simulation alone, open loop and closed loop (latency kernel)
#   rcp          tools/probe/rcp_probe: v_rcp_f64 accuracy and one- vs two-step correctly rounded division
#   handoff      tools/probe/handoff: dependent hand-off latency between two waves
#   tworank      bench.py --gpus 2 with both ranks on card 0 (gloo)
#   sweep        tools/relax/sweep_bench: one relaxation sweep's phases L and F on the GPU, W = 1,024 and 4,096
#                (inputs from tools/relax/make_sweeps.sh), plus its rocprofv3 kernel stats
#   tworank_parity  the same with each rank's reference parity processes and the job-level roofline
#   regions_single  lone-wave region profiles of the shipped compiled-configuration latency kernel
#                (-DPU_PROF through PRIMEUNCORE_JIT_EXTRA), open and closed loop
#   regions_ens  the same for the throughput kernel at the headline's replica count
#   ab_modes:V1,V2,...   interleaved same-box A/B of engine libraries (main = libprimeuncore.so, else
#                libprimeuncore_V.so; V@FLAGS also sets PRIMEUNCORE_JIT_EXTRA=FLAGS, '+' for a space
#                (compiled by hipRTC on the box unless warmed in-tree first:
#                PRIMEUNCORE_JIT_EXTRA=FLAGS python3 tools/jit_warm.py --only "preset C4"),
#                and V#W sets PRIMEUNCORE_JIT_WAVES=W) in three regimes: headline, one simulation
#                alone open / closed loop
#   ab_single:V1,V2,...  the same, one simulation alone only
#   ab_ens:V1,V2,...     the same, headline only (3 rounds)
#   ab_c3:V1,V2,...      the same on bench --config C3 (2 rounds)
#   ab_ensc:V1,V2,...    headline open loop and the same workload closed loop (2 rounds)
#   ab_driver:V1,V2,...  the headline on the driver's window (--steps 20 --warmup 5), 2 interleaved rounds
#   refwrap      tools/ref_overhead.py: the reference CPU uncore with and without the golden counting wraps
#   residency    tools/probe/residency: one-wave workgroups resident per CU by resource shape
#   diag:V       one headline run (5+5 steps) of variant V (ab syntax) with its bench log kept
#   ab_pool      headline with the replica pool (--spare-replicas 0.1) vs without (0), 3 interleaved rounds
set -o pipefail
T=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/${T}
BENCH="python bench.py"
DRIVER="--steps 20 --warmup 5"

variant_env() {   # V[#WAVES][@FLAGS][^NAME=VALUE]: library V (main = the product), compiled-configuration
  local v=$1 lib extra waves kv   # options, one more environment variable
  case $v in *^*) kv=${v#*^}; v=${v%%^*}; export "${kv%%=*}=${kv#*=}";; esac
  lib=${v%%[@#]*}
  case $v in *@*) extra=${v#*@}; export PRIMEUNCORE_JIT_EXTRA="${extra//+/ }";; esac
  case $v in *#*) waves=${v#*#}; waves=${waves%%@*}; export PRIMEUNCORE_JIT_WAVES=$waves;; esac
  if [ "$lib" != main ]; then export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_$lib.so; fi
}

ab() {   # ab ROUNDS MODES VARIANTS
  local R=$1 MODES=$2 VARS=$3 mode v ARGS
  for i in $(seq 1 "$R"); do
    for mode in $MODES; do
      case $mode in
        ens) ARGS="--steps 5 --warmup 5 --no-cpu --no-extras";;
        c3) ARGS="--config C3 --steps 5 --warmup 5 --no-cpu --no-extras";;
        ensc) ARGS="--steps 5 --warmup 5 --no-cpu --no-extras --replay closed";;
        c5) ARGS="--config C5 --steps 5 --warmup 5 --no-cpu --no-extras";;
        single) ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras";;
        closed) ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras --replay closed";;
      esac
      for v in ${VARS//,/ }; do
        ( variant_env "$v"
          timeout -k 10 200 $BENCH $ARGS 2>>${O}_ab.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); v=b['value']; print('$mode', '$v', round(v) if v < 1e6 else round(v / 1e6, 2), flush=True)" ) || return 1
      done
    done
  done
}

for S in "$@"; do
  echo "[gpu_session] $T: $S ($(date +%T))"
  case $S in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > ${O}_gpu_tests.log 2>&1 || exit 1;;
    latency) timeout -k 10 300 python tools/latency_bench.py --calls 2000 --out ${O}_latency.json > ${O}_latency.log 2>&1 || exit 1;;
    smoke) timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || exit 1;;
    traffic) timeout -k 10 500 python tools/pmc_traffic.py --work /tmp/pmc --out ${O}_traffic.json -- $DRIVER --no-cpu --no-extras > ${O}_traffic.log 2>&1 || exit 1;;
    bench) TJ=""; [ -f ${O}_traffic.json ] && TJ="--traffic-json ${O}_traffic.json"
           timeout -k 10 400 $BENCH $DRIVER $TJ > ${O}_bench.json 2> ${O}_bench.log || exit 1;;
    bench_c3) timeout -k 10 500 $BENCH --config C3 $DRIVER > ${O}_bench_c3.json 2> ${O}_bench_c3.log || exit 1;;
    bench_c5) timeout -k 10 600 $BENCH --config C5 $DRIVER > ${O}_bench_c5.json 2> ${O}_bench_c5.log || exit 1;;
    bench_default) timeout -k 10 400 $BENCH > ${O}_bench_default.json 2> ${O}_bench_default.log || exit 1;;
    rocprof) TJ=""; [ -f ${O}_traffic.json ] && TJ="--traffic-json ${O}_traffic.json"
             timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_prof -o run -- python3 bench.py $DRIVER --no-cpu --no-extras $TJ > ${O}_bench_under_rocprof.json 2> ${O}_rocprof.log || exit 1
             cp /tmp/${T}_prof/run_kernel_stats.csv ${O}_kernel_stats.csv || exit 1;;
    sq) timeout -k 10 700 python tools/pmc_sq.py --work /tmp/pmc_sq --out ${O}_sq.json -- --steps 3 --warmup 5 --no-cpu --no-extras > ${O}_sq.log 2>&1 || exit 1;;
    sq_closed) timeout -k 10 700 python tools/pmc_sq.py --work /tmp/pmc_sqc --out ${O}_sq_closed.json -- --steps 3 --warmup 5 --no-cpu --no-extras --replay closed > ${O}_sq_closed.log 2>&1 || exit 1;;
    traffic_closed) timeout -k 10 500 python tools/pmc_traffic.py --work /tmp/pmcc --out ${O}_traffic_closed.json -- $DRIVER --no-cpu --no-extras --replay closed > ${O}_traffic_closed.log 2>&1 || exit 1;;
    regions_closed) timeout -k 10 300 python tools/prof_regions.py --jit -- --steps 3 --warmup 5 --no-cpu --no-extras --replay closed > ${O}_regions_closed.txt 2>&1 || exit 1;;
    sq_single) timeout -k 10 500 python tools/pmc_sq.py --kernel pu_jit_uncore_s1_h1 --work /tmp/pmc_sq1 --out ${O}_sq_single_open.json -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > ${O}_sq_single_open.log 2>&1 || exit 1
               timeout -k 10 500 python tools/pmc_sq.py --kernel pu_jit_uncore_s1_h1 --work /tmp/pmc_sq2 --out ${O}_sq_single_closed.json -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras --replay closed > ${O}_sq_single_closed.log 2>&1 || exit 1;;
    rcp) timeout -k 10 120 tools/probe/rcp_probe 4096 > ${O}_rcp.json 2> ${O}_rcp.log || exit 1;;
    handoff) timeout -k 10 120 tools/probe/handoff > ${O}_handoff.json 2> ${O}_handoff.log || exit 1;;
    tworank) PU_BENCH_DEVICE=0 timeout -k 10 300 $BENCH --gpus 2 --steps 3 --warmup 2 --no-cpu --dist-backend gloo > ${O}_two_rank.json 2> ${O}_two_rank.log || exit 1;;
    tworank_parity) PU_BENCH_DEVICE=0 timeout -k 10 400 $BENCH --gpus 2 --steps 3 --warmup 2 --dist-backend gloo > ${O}_two_rank_parity.json 2> ${O}_two_rank_parity.log || exit 1;;
    sweep) for W in 1024 4096; do
             timeout -k 10 120 tools/relax/sweep_bench tools/relax/data/w$W 200 > ${O}_sweep_w$W.json 2> ${O}_sweep_w$W.log || exit 1
           done
           timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_sweep -o run -- tools/relax/sweep_bench tools/relax/data/w4096 50 > ${O}_sweep_w4096_rocprof.json 2> ${O}_sweep_rocprof.log || exit 1
           cp /tmp/${T}_sweep/run_kernel_stats.csv ${O}_sweep_kernel_stats.csv || exit 1;;
    regions_single)
      timeout -k 10 200 python tools/prof_regions.py --jit -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > ${O}_regions_single_open.txt 2>&1 || exit 1
      timeout -k 10 200 python tools/prof_regions.py --jit -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras --replay closed > ${O}_regions_single_closed.txt 2>&1 || exit 1;;
    regions_ens)
      timeout -k 10 300 python tools/prof_regions.py --jit -- --steps 3 --warmup 5 --no-cpu --no-extras > ${O}_regions_ens.txt 2>&1 || exit 1;;
    refwrap) timeout -k 10 200 python tools/ref_overhead.py --seconds 5 --rounds 3 --json ${O}_ref_overhead.json > ${O}_ref_overhead.log 2>&1 || exit 1;;
    residency) timeout -k 10 120 tools/probe/residency > ${O}_residency.json 2> ${O}_residency.log || exit 1;;
    diag:*) ( variant_env "${S#diag:}"
              timeout -k 10 300 $BENCH --steps 5 --warmup 5 --no-cpu --no-extras > ${O}_diag.json 2> ${O}_diag.log ) || exit 1;;
    ab_modes:*) ab 2 "ens single closed" "${S#ab_modes:}" > ${O}_ab_modes.txt || exit 1;;
    ab_single:*) ab 2 "single closed" "${S#ab_single:}" > ${O}_ab_single.txt || exit 1;;
    ab_ens:*) ab 3 "ens" "${S#ab_ens:}" > ${O}_ab_ens.txt || exit 1;;
    ab_c3:*) ab 2 "c3" "${S#ab_c3:}" > ${O}_ab_c3.txt || exit 1;;
    ab_ensc:*) ab 2 "ens ensc" "${S#ab_ensc:}" > ${O}_ab_ensc.txt || exit 1;;
    ab_driver:*) for i in 1 2; do for v in $(echo "${S#ab_driver:}" | tr ',' ' '); do
               ( variant_env "$v"
                 timeout -k 10 400 $BENCH $DRIVER --no-cpu --no-extras 2>>${O}_ab.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=b['config']; p=c.get('replica_pool') or {}; print('driver', '$v', round(b['value']/1e6,2), 'M/s', 'replicas', c['replicas_per_gpu'], 'slots', c['wavefronts_per_gpu'], 'halted', c['halted_replicas'], 'busy', round(p.get('busy_fraction', 0), 4), 'started', p.get('replicas_started'), flush=True)" >> ${O}_ab_driver.txt ) || exit 1
             done; done;;
    ab_pool) for i in 1 2 3; do for sp in 0.1 0; do
               timeout -k 10 300 $BENCH $DRIVER --no-cpu --no-extras --spare-replicas $sp 2>>${O}_ab.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=b['config']; p=c.get('replica_pool') or {}; print('spare $sp', round(b['value']/1e6,2), 'M/s', 'replicas', c['replicas_per_gpu'], 'halted', c['halted_replicas'], 'busy', round(p.get('busy_fraction', 0), 4), flush=True)" >> ${O}_ab_pool.txt || exit 1
             done; done;;
    *) echo "unknown step $S"; exit 2;;
  esac
done
du -sh gpurun_out
exit 0
