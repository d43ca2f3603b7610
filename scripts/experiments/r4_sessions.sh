# Round-4 GPU-box sessions, one function per session:
#   bash scripts/experiments/r4_sessions.sh <session>
# Each writes under gpurun_out/r4_<session>/. The summaries were copied into
# the profile directory named in the comment (see scripts/README.md).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=${1:?usage: r4_sessions.sh <session>}
O=gpurun_out/r4_$S
mkdir -p "$O"

step() {  # step <name> <timeout> <cmd...>: a crash, abort or timeout ends the session
  local name=$1 t=$2
  shift 2
  echo "=== $name ($(date +%T))"
  local t0
  t0=$(date +%s.%N)
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc wall_s=$(python3 -c "print(round($(date +%s.%N)-$t0,1))")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "fatal rc=$rc in $name: stopping"
    exit $rc
  fi
  return 0
}

irq_map() {  # which CPUs the GPU's interrupt vectors are routed to
  python3 - <<'EOF' > "$O/irq_map.txt" 2>&1
import os, re
for line in open("/proc/interrupts"):
    if "amdgpu" in line or "kfd" in line:
        irq = line.split(":")[0].strip()
        try:
            aff = open(f"/proc/irq/{irq}/effective_affinity_list").read().strip()
        except OSError:
            aff = "?"
        print(irq, "effective_cpus", aff, " ".join(line.split()[-3:]))
EOF
}

case "$S" in
recvcost)  # profiles/r4_recvcost: headline vs no-DMA vs host-read vs discard baseline, with and without GPU interrupts
  irq_map
  step default 400 python3 -u scripts/experiments/recv_cost_ab.py --tag default
  step noint 400 env HSA_ENABLE_INTERRUPT=0 python3 -u scripts/experiments/recv_cost_ab.py --tag noint
  step default2 400 python3 -u scripts/experiments/recv_cost_ab.py --tag default2 --reps 2
  ;;
recvcost2)  # profiles/r4_recvcost/after_listener_cc: the same A/B once the endpoint's listener carries its CC, + a full bench
  step pytest_sink 300 python3 -u -m pytest tests/test_gpu_sink.py tests/test_gpu_crc32c.py -x -q --timeout 120 --timeout-method thread
  step ab 400 python3 -u scripts/experiments/recv_cost_ab.py --tag listener_cc --variants head,head_wc,head_4m,head_refill,head_spin,nodma,hostread,base
  step mux 400 python3 -u scripts/experiments/mux_fair_ab.py
  step bench 600 python3 bench.py --json-out "$O/bench.json"
  step diag100 400 python3 bench.py --steps 100 --warmup 3 --side-steps 0 --read-diag --json-out "$O/diag100.json"
  for k in 1 2; do
    for p in share_quota split_quota; do
      step "http_${p}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default,ref_default_100m \
        --ref-http-placement $p --json-out "$O/http_${p}_$k.json"
    done
  done
  ;;
main4)  # the round-4 GPU checkpoint: GPU suite, recv-cost A/B, full bench, 100-read diag, mux + HTTP placement A/Bs
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step ab 400 python3 -u scripts/experiments/recv_cost_ab.py --tag main4 \
    --variants head,head_wc,head_4m,head_refill,head_spin,nodma,hostread,base
  step bench 600 python3 bench.py --json-out "$O/bench.json"
  step diag100 400 python3 bench.py --steps 100 --warmup 3 --side-steps 0 --read-diag --json-out "$O/diag100.json"
  step mux 400 python3 -u scripts/experiments/mux_fair_ab.py
  for k in 1 2; do
    for p in share_quota split_quota; do
      step "http_${p}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default,ref_default_100m \
        --ref-http-placement $p --json-out "$O/http_${p}_$k.json"
    done
  done
  ;;
main5)  # send scheduler on the GPU box; recv-cost A/B with more reps; two benches; the CLI soak
  step pytest_sink 300 python3 -u -m pytest tests/test_gpu_sink.py tests/test_gpu_crc32c.py -x -q --timeout 120 --timeout-method thread
  step mux 400 python3 -u scripts/experiments/mux_fair_ab.py --quanta 0,1024
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag main5 --reps 5 \
    --variants head,head_4x2,head_spin,nodma,hostread,base
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  step soak 900 python3 -u scripts/soak.py --out "$O/soak" --duration 120s
  ;;
main6)  # ring footprint sweep; endpoint quantum at 48 streams; two benches
  step ab 600 python3 -u scripts/experiments/recv_cost_ab.py --tag main6 --reps 4 \
    --variants head,head_4x2,head_3x2,head_2x2,head_4x1m,head_8x512k,head_wc,head_4x2_wc,nodma,base
  step mux 400 python3 -u scripts/experiments/mux_fair_ab.py --quanta 0,256,64 --reps 3
  step bench1 600 python3 bench.py --slots 4 --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  ;;
main7)  # bounce receive (VERDICT r3 next #1b) against the direct ring, nodma and the baseline
  # (ring_bounce was removed after this session, profiles/r4_recvcost; the variants below no longer exist)
  step pytest_bounce 300 python3 -u -m pytest tests/test_gpu_sink.py -x -q --timeout 120 --timeout-method thread -k "bounce or wc or byte_exact"
  step ab 600 python3 -u scripts/experiments/recv_cost_ab.py --tag main7 --reps 5 \
    --variants head,head_2x2,head_4x1m,head_bounce,head_bounce_4x2,head_bounce2,nodma,base
  step mux 300 python3 -u scripts/experiments/mux_fair_ab.py --quanta 0 --leads 0,64,16 --reps 3
  step bench1 600 python3 bench.py --ring-bounce on --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --slots 4 --json-out "$O/bench2.json"
  ;;
main8)  # small ring footprints (main6/main7: 4 MiB rings read 4-9% faster than 16 MiB); bench on 4 x 1 MiB
  step ab 600 python3 -u scripts/experiments/recv_cost_ab.py --tag main8 --reps 5 \
    --variants head,head_4x1m,head_3x1m,head_2x1m,head_6x1m,head_4x512k,head_8x256k,nodma,base
  step bench1 600 python3 bench.py --slot-bytes 1MiB --slots 4 --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  step bench3 600 python3 bench.py --slot-bytes 1MiB --slots 4 --json-out "$O/bench3.json"
  ;;
main9)  # round-4 checkpoint on the 4 x 1 MiB default: GPU suite, smoke, A/B (submitter polling at 1 MiB
  # slots), two benches, one bench under rocprofv3 --kernel-trace --stats, 100-read diag
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag main9 --reps 5 \
    --variants head_4x1m,head_4x1m_spin,head_3x1m,head,nodma,base
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  step prof 600 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 bench.py --steps 20 --warmup 3 \
    --blocks ceiling --json-out "$O/bench_prof.json"
  step diag100 400 python3 bench.py --steps 100 --warmup 3 --side-steps 0 --read-diag --json-out "$O/diag100.json"
  ;;
crcw)  # slot CRC kernel on 1 MiB slots inside the read pipeline: waves per workgroup
  for w in 1 2 4 8; do
    step "prof_w$w" 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_w$w" -o run -- python3 bench.py --steps 20 \
      --warmup 3 --blocks ceiling --crc-slot-waves $w --json-out "$O/bench_w$w.json"
  done
  ;;
refring)  # 48 workers x 100 MiB into HBM: per-worker ring footprint (the multiplexed reader's copy destinations)
  for k in 1 2; do
    for r in 2x2MiB 4x256KiB 2x512KiB 4x512KiB; do
      step "ref_${r}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default_100m --ref-gpu-ring $r \
        --json-out "$O/ref_${r}_$k.json"
    done
  done
  ;;
muxiso)  # the multiplexed gRPC reader on a core of its own, after the pacing fix (r3: mixed)
  for k in 1 2 3; do
    for m in shared isolate; do
      step "mux_${m}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default,ref_default_100m,list_read \
        --mux-reader $m --json-out "$O/mux_${m}_$k.json"
    done
  done
  ;;
bigring)  # one stream into the multiplexed reader's footprint: does a 48-96 MiB ring cost the copy 2x?
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag bigring --reps 3 \
    --variants head_4x1m,head,head_24x2,head_48x2,nodma_48x2,nodma
  ;;
connring)  # the connection ring: GPU tests, then the multiplexed GPU blocks with it on / off
  step pytest_ring 300 python3 -u -m pytest tests/test_gpu_conn_ring.py -x -v --timeout 120 --timeout-method thread
  for k in 1 2; do
    for c in on off; do
      step "ring_${c}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default_100m,list_read \
        --conn-ring $c --json-out "$O/ring_${c}_$k.json"
    done
  done
  ;;
ringgeom)  # connection-ring geometry for the 48 x 100 MiB gRPC -> HBM block and config-3 list-read
  for k in 1 2; do
    for c in 8x1MiB 4x1MiB 16x1MiB 8x2MiB 4x2MiB off; do
      step "geom_${c}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default_100m,list_read \
        --conn-ring $c --json-out "$O/geom_${c}_$k.json"
    done
  done
  ;;
final1)  # checkpoint on the final round-4 defaults (4 x 1 MiB headline ring, connection ring): GPU suite,
  # smoke, two benches, the 8-rank rehearsal on one GPU (gloo), a 60 s soak per protocol
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  t0=$(date +%s.%N)
  export GCSB_DIST_BACKEND=gloo
  step rehearsal8 400 python3 bench.py --gpus 8 --object-size 64MiB --steps 5 --side-steps 3 \
    --json-out "$O/rehearsal8.json"
  unset GCSB_DIST_BACKEND
  python3 -c "print('rehearsal8 wall_s', round($(date +%s.%N)-$t0, 1))" > "$O/rehearsal8_wall.txt"
  step soak 600 python3 -u scripts/soak.py --out "$O/soak" --duration 60s --metrics-interval 20s
  ;;
span)  # receive windows spanning two free slots of the contiguous ring (fewer recv calls) vs stopping at each slot
  step pytest_sink 400 python3 -u -m pytest tests/test_gpu_sink.py tests/test_gpu_conn_ring.py tests/test_gpu_large_object.py \
    -x -q --timeout 120 --timeout-method thread
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag span --reps 5 \
    --variants head_4x1m,head_4x1m_nospan,head_8x512k,head_8x512k_nospan,nodma,base
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  ;;
handoff)  # how much of the receiving thread the slot hand-off takes (GpuSinkStats::handoff_s)
  step ab 400 python3 -u scripts/experiments/recv_cost_ab.py --tag handoff --reps 3 \
    --variants head_4x1m,head,nodma,base
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  ;;
pfw)  # PREFETCHW over the next receive window (re-own the lines the copy engine read); the option was
  # removed after this session (profiles/r4_recvcost), the pfw variants no longer exist
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag pfw --reps 5 \
    --variants head_4x1m,head_4x1m_pfw256k,head_4x1m_pfw1m,nodma,base
  ;;
final2)  # checkpoint after span / handoff counters / stat resets: GPU suite, smoke, two benches
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  ;;
lag)  # submit a filled slot one slot later (the copy engine reads L3 lines, not the receiving core's L2);
  # submit_lag was removed after this session (profiles/r4_recvcost), the lag variants no longer exist
  step pytest_lag 300 python3 -u -m pytest tests/test_gpu_sink.py -x -q --timeout 120 --timeout-method thread
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag lag --reps 5 \
    --variants head_4x1m,head_4x1m_lag,head_6x512k_lag,nodma,base
  ;;
refpair)  # 48 x 100 MiB gRPC: the one connection's reader + the endpoint on a core pair each (GPU sink: the
  # workers only wait) against one L3 domain
  for k in 1 2; do
    for m in same pair; do
      step "rp_${m}_$k" 300 python3 bench.py --steps 5 --warmup 1 --blocks ref_default_100m,ref_default \
        --ref-grpc-placement $m --json-out "$O/rp_${m}_$k.json"
    done
  done
  ;;
final3)  # last checkpoint of the round: GPU suite, smoke, two benches, the 8-rank rehearsal
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  t0=$(date +%s.%N)
  export GCSB_DIST_BACKEND=gloo
  step rehearsal8 400 python3 bench.py --gpus 8 --object-size 64MiB --steps 5 --side-steps 3 \
    --json-out "$O/rehearsal8.json"
  unset GCSB_DIST_BACKEND
  python3 -c "print('rehearsal8 wall_s', round($(date +%s.%N)-$t0, 1))" > "$O/rehearsal8_wall.txt"
  ;;
evidence)  # final-code evidence: 100-read stall attribution (off-core sampler), kernel + copy trace of the headline
  step diag100 400 python3 bench.py --steps 100 --warmup 3 --side-steps 0 --read-diag --json-out "$O/diag100.json"
  step prof 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d "$O/prof" -o run -- python3 bench.py \
    --steps 20 --warmup 3 --blocks ceiling --json-out "$O/bench_prof.json"
  ;;
softnet)  # do the loopback retransmits follow input-backlog drops? two 100-read diag runs
  step diag100a 400 python3 bench.py --steps 100 --warmup 3 --side-steps 0 --read-diag --json-out "$O/diag100a.json"
  step diag100b 400 python3 bench.py --steps 100 --warmup 3 --side-steps 0 --read-diag --json-out "$O/diag100b.json"
  ;;
twocore)  # the headline's receiving thread on the baseline's two cores vs its own core pair
  step ab 500 python3 -u scripts/experiments/recv_cost_ab.py --tag twocore --reps 6 \
    --variants head_4x1m,head_4x1m_2core,nodma,base
  ;;
crc8)  # slot CRC kernel: slice-by-8 tables (half the L2-cold LDS stage) vs slice-by-16, in the read pipeline
  step pytest_crc 300 python3 -u -m pytest tests/test_gpu_crc32c.py -x -q --timeout 120 --timeout-method thread
  for k in 1 2; do
    for c in off on; do
      step "prof_s8${c}_$k" 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_s8${c}_$k" -o run -- python3 \
        bench.py --steps 20 --warmup 3 --blocks ceiling --crc-slice8 $c --json-out "$O/bench_s8${c}_$k.json"
    done
  done
  ;;
final4)  # after slice-by-8 by default: GPU suite, smoke, two benches
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  ;;
dist)  # the HEAD headline against its bracketing baseline, eight back-to-back runs (distribution of vs_baseline)
  for k in 1 2 3 4 5 6 7 8; do
    step "b_$k" 300 python3 bench.py --blocks cpu_baseline,ceiling --json-out "$O/b_$k.json"
  done
  ;;
final5)  # after the receiver-interference field: smoke, two full benches, four more headline runs
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench1 600 python3 bench.py --json-out "$O/bench1.json"
  step bench2 600 python3 bench.py --json-out "$O/bench2.json"
  for k in 1 2 3 4; do
    step "h_$k" 300 python3 bench.py --blocks cpu_baseline,ceiling --json-out "$O/h_$k.json"
  done
  ;;
final6)  # closing check of HEAD: GPU suite, smoke, the driver's bench command
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench 600 python3 bench.py --json-out "$O/bench.json"
  ;;
clock)  # the placement cores' clock through every block (sysdiag.ClockSampler): one full bench, six headline runs
  step bench 600 python3 bench.py --json-out "$O/bench.json"
  for k in 1 2 3 4 5 6; do
    step "h_$k" 300 python3 bench.py --blocks cpu_baseline,ceiling --json-out "$O/h_$k.json"
  done
  ;;
dist2)  # headline vs its bracketing baseline, interleaved: pair (default) against pair2 (a second quiet core each)
  for k in 1 2 3 4 5 6 7 8; do
    step "pair_$k" 300 python3 bench.py --blocks cpu_baseline,ceiling --json-out "$O/pair_$k.json"
    step "pair2_$k" 300 python3 bench.py --blocks cpu_baseline,ceiling --affinity pair2 --json-out "$O/pair2_$k.json"
  done
  ;;
soak)  # profiles/r4_soak: execute_pb.sh with 48 workers x 100 MiB, -sink gpu, 120 s per protocol, exporter at 30 s
  step soak 900 python3 -u scripts/soak.py --out "$O" --duration 120s
  ;;
*)
  echo "unknown session $S"
  exit 2
  ;;
esac
