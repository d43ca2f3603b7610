# Round-3 GPU-box sessions, one function per session:
#   bash scripts/experiments/r3_sessions.sh <session>
# Each writes under gpurun_out/r3_<session>/. The summaries were copied into
# the profile directory named in the comment (see scripts/README.md).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=${1:?usage: r3_sessions.sh <session>}
O=gpurun_out/r3_$S
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

case "$S" in
wccheck)  # profiles/r3_ring_thp/wc: the write-combined list-read default, GPU sink tests + list-read runs
  step pytest_sink 300 python3 -u -m pytest tests/test_gpu_sink.py -x -q --timeout 120 --timeout-method thread
  for k in 1 2 3; do
    for v in on off; do
      step "l${v}_$k" 300 python3 bench.py --steps 20 --warmup 3 --blocks list_read --list-ring-wc $v \
        --json-out "$O/l${v}_$k.json"
    done
  done
  ;;
ringwc)  # profiles/r3_ring_thp/wc: read-sink rings in write-combined memory (GCSB_RING_WC) vs THP cached
  for k in 1 2 3; do
    for v in 0 1; do
      step "w${v}_$k" 300 env GCSB_RING_WC=$v python3 bench.py --steps 20 --warmup 3 \
        --blocks cpu_baseline,list_read,ceiling --json-out "$O/w${v}_$k.json"
    done
  done
  ;;
slotreuse)  # profiles/r3_twins/slotreuse: the receiving thread's time reusing ring slots (event wait + harvest)
  for k in 1 2 3; do
    step "u_$k" 300 python3 bench.py --steps 20 --warmup 3 --blocks ceiling --json-out "$O/u_$k.json"
  done
  ;;
bracket)  # profiles/r3_twins/bracket: the two-core baseline before AND after the headline (drift cancels)
  for k in 1 2 3 4 5; do
    step "k_$k" 300 python3 bench.py --steps 20 --warmup 3 --baseline-bracket on --blocks cpu_baseline,ceiling \
      --json-out "$O/k_$k.json"
  done
  ;;
rehearse)  # profiles/r3_rehearsal8/head: gloo rehearsals at 2, 4 and 8 ranks on one GPU with every round-3 default
  for n in 2 4 8; do
    step "rehearsal$n" 500 env GCSB_DIST_BACKEND=gloo python3 bench.py --gpus $n --object-size 64MiB --steps 5 \
      --side-steps 3 --json-out "$O/rehearsal$n.json"
  done
  ;;
long)  # profiles/r3_final/long: 100 timed reads per run (p99 is no longer the maximum) + a kernel/copy profile at HEAD
  for k in 1 2 3; do
    step "long_$k" 300 python3 bench.py --steps 100 --warmup 5 --blocks ceiling --json-out "$O/long_$k.json"
  done
  step rocprof 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof" -o bench -- \
    python3 bench.py --steps 20 --warmup 3
  ;;
ringalloc)  # profiles/r3_ring_thp/alloc: ring from THP + hipHostRegister vs hipHostMalloc, against the two-core baseline
  for k in 1 2 3; do
    for v in thp hip; do
      step "a${v}_$k" 300 env GCSB_RING_ALLOC=$v python3 bench.py --steps 20 --warmup 3 \
        --blocks cpu_baseline,ceiling --json-out "$O/a${v}_$k.json"
    done
  done
  ;;
ringsmall2)  # profiles/r3_ring_thp/small2: ring reuse distance against the two-core baseline, more reps
  for k in 1 2 3 4; do
    for v in 8x2MiB 2x2MiB 2x1MiB; do
      n=${v%x*}; b=${v#*x}
      step "r${v}_$k" 300 python3 bench.py --steps 20 --warmup 3 --slots $n --slot-bytes $b \
        --blocks cpu_baseline,ceiling --json-out "$O/r${v}_$k.json"
    done
  done
  ;;
ringsmall)  # profiles/r3_ring_thp/small: small headline rings (reuse distance) against the two-core baseline
  for k in 1 2 3; do
    for v in 8x2MiB 4x2MiB 3x2MiB 2x2MiB; do
      n=${v%x*}; b=${v#*x}
      step "r${v}_$k" 300 python3 bench.py --steps 20 --warmup 3 --slots $n --slot-bytes $b \
        --blocks cpu_baseline,ceiling --json-out "$O/r${v}_$k.json"
    done
  done
  ;;
base2core)  # profiles/r3_twins/base2core: the reference-semantics baseline on the client + submitter cores
  for k in 1 2 3; do
    step "b_$k" 300 python3 bench.py --steps 20 --warmup 3 --blocks cpu_baseline,ceiling --json-out "$O/b_$k.json"
  done
  ;;
spincubic)  # profiles/r3_refill/spin: submitter polls before sleeping (no futex wake per slot on the reader), cubic
  for k in 1 2 3 4; do
    for v in 0 100; do
      step "s${v}_$k" 300 env GCSB_SUBMIT_SPIN_US=$v python3 bench.py --steps 20 --warmup 3 --blocks ceiling \
        --json-out "$O/s${v}_$k.json"
    done
  done
  ;;
crcwaves)  # profiles/r3_crc_waves: slot kernel waves per workgroup inside the read pipeline (L2-cold tables)
  for w in 2 4 8 1; do
    step "prof_w$w" 300 env GCSB_CRC_SLOT_WAVES=$w rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$O/prof_w$w" -o b -- python3 bench.py --steps 20 --warmup 3 --blocks ceiling
  done
  ;;
refill)  # profiles/r3_refill: a payload recvmsg() that also refills the header buffer (GCSB_RECV_REFILL) vs not
  for k in 1 2 3; do
    for v in 0 1; do
      step "f${v}_$k" 300 env GCSB_RECV_REFILL=$v python3 bench.py --steps 20 --warmup 3 \
        --blocks compare,list_read,ceiling --json-out "$O/f${v}_$k.json"
    done
  done
  ;;
ringcubic)  # profiles/r3_ring_thp/cubic: headline ring geometry with cubic endpoint sockets (bigger recv asks)
  for k in 1 2 3; do
    for v in 8x2MiB 4x4MiB 2x8MiB 4x2MiB; do
      n=${v%x*}; b=${v#*x}
      step "r${v}_$k" 300 python3 bench.py --steps 20 --warmup 3 --slots $n --slot-bytes $b --blocks ceiling \
        --json-out "$O/r${v}_$k.json"
    done
  done
  ;;
cc)  # profiles/r3_twins/cc: endpoint congestion control and connection age, HTTP one stream (compare) + headline
  { cat /proc/sys/net/ipv4/tcp_congestion_control /proc/sys/net/ipv4/tcp_allowed_congestion_control \
      /proc/sys/net/ipv4/tcp_available_congestion_control; } > "$O/env.txt" 2>&1
  for k in 1 2; do
    for v in default reno bbr cubic; do
      cc=$v; [ "$v" = default ] && cc=
      step "c${v}_$k" 300 env GCSB_SRV_CC=$cc python3 bench.py --steps 20 --warmup 3 --blocks compare,ceiling \
        --json-out "$O/c${v}_$k.json"
    done
  done
  ;;
pair2)  # profiles/r3_ring_thp/pair2: headline placement, one core each vs two cores each (tails)
  for k in 1 2 3 4; do
    for a in pair pair2; do
      step "a${a}_$k" 300 python3 bench.py --steps 20 --warmup 3 --affinity $a --blocks ceiling \
        --json-out "$O/a${a}_$k.json"
    done
  done
  ;;
refplace)  # profiles/r3_mux_thp/refplace: 48-worker gRPC placement (share_quota vs one L3 domain vs share)
  for k in 1 2 3; do
    for m in share_quota same share; do
      step "p${m}_$k" 300 python3 bench.py --steps 20 --warmup 3 --blocks ref_default --ref-grpc-placement $m \
        --json-out "$O/p${m}_$k.json"
    done
  done
  ;;
slicering)  # profiles/r3_ring_thp/sliced: sliced-read ring per sink (2 sinks per stream), THP endpoint
  for k in 1 2 3; do
    for r in 8x2MiB 4x1MiB 2x2MiB 4x2MiB; do
      n=${r%x*}; b=${r#*x}
      step "s${r}_$k" 300 python3 bench.py --steps 20 --warmup 3 --blocks sliced --sliced-slots $n \
        --sliced-slot-bytes $b --json-out "$O/s${r}_$k.json"
    done
  done
  ;;
sndbuf)  # profiles/r3_twins/sndbuf: HTTP / gRPC one-stream read by endpoint send buffer (autotuned vs explicit)
  for rep in 1 2; do
    for v in 0 33554432 8388608; do
      step "bench_s${v}_r$rep" 300 env GCSB_RECV_DIAG=1 GCSB_SRV_SNDBUF=$v python3 bench.py --steps 20 --warmup 3 \
        --blocks compare,ceiling --json-out "$O/bench_s${v}_r$rep.json"
    done
  done
  ;;
httppiece)  # profiles/r3_twins/http_piece: HTTP one-stream read, endpoint send call size
  for rep in 1 2; do
    for v in 8388608 2097152 1048576 16777216; do
      step "bench_p${v}_r$rep" 300 env GCSB_RECV_DIAG=1 GCSB_SRV_HTTP_PIECE=$v python3 bench.py --steps 20 --warmup 3 \
        --protocol http --blocks ceiling --json-out "$O/bench_p${v}_r$rep.json"
    done
  done
  ;;
twins)  # profiles/r3_twins: per-thread CPU of the headline's HTTP / reference-semantics twins
  for rep in 1 2; do
    step "bench_r$rep" 300 env GCSB_RECV_DIAG=1 python3 bench.py --steps 20 --warmup 3 \
      --blocks cpu_baseline,compare --json-out "$O/bench_r$rep.json"
  done
  ;;
check8thp)  # profiles/r3_rehearsal8/thp, r3_final/prof: 8-rank gloo rehearsal and a kernel profile with the THP endpoint
  step rehearsal8 500 env GCSB_DIST_BACKEND=gloo python3 bench.py --gpus 8 --object-size 64MiB --steps 5 --side-steps 3
  step rocprof 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof" -o bench -- \
    python3 bench.py --steps 10 --warmup 2
  ;;
ringthp)  # profiles/r3_ring_thp: headline ring geometry with the THP source (receiver-bound now)
  for rep in 1 2 3; do
    for v in 8x2MiB 4x2MiB 8x1MiB 16x2MiB; do
      n=${v%x*}; b=${v#*x}
      step "bench_${v}_r$rep" 300 python3 bench.py --steps 20 --warmup 3 --slots $n --slot-bytes $b \
        --blocks ceiling --json-out "$O/bench_${v}_r$rep.json"
    done
  done
  ;;
muxiso)  # profiles/r3_mux_thp/isolate: multiplexed reader on its own core vs shared, THP source
  for rep in 1 2 3; do
    for v in shared isolate; do
      step "bench_${v}_r$rep" 300 python3 bench.py --steps 20 --warmup 3 --mux-reader $v \
        --blocks list_read,ref_default --json-out "$O/bench_${v}_r$rep.json"
    done
  done
  ;;
muxdiag)  # profiles/r3_mux_thp: multiplexed reader with the THP source, recv() wall time inside DATA dispatch
  for rep in 1 2; do
    step "bench_diag_r$rep" 300 env GCSB_RECV_DIAG=1 python3 bench.py --steps 20 --warmup 3 \
      --blocks list_read,ref_default --json-out "$O/bench_diag_r$rep.json"
  done
  ;;
thpsend)  # profiles/r3_thp_send: endpoint sends synthetic bodies by vmsplice from THP vs sendfile from the memfd
  for rep in 1 2; do
    for v in sendfile vmsplice; do
      step "bench_${v}_r$rep" 300 env GCSB_SRV_SEND=$v python3 bench.py --steps 20 --warmup 3 \
        --json-out "$O/bench_${v}_r$rep.json"
    done
  done
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  ;;
thpsrc)  # profiles/r3_splice: receiver cost by the sender's page size (4 KiB page cache vs THP)
  { uname -r; cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/shmem_enabled;
    grep -i huge /proc/meminfo; } > "$O/env.txt" 2>&1
  P=custom_go_client_benchmark_amd/bin/splice_probe
  for rep in 1 2; do
    for src in memfd anon_thp memfd_thp; do
      for st in 1 8; do
        step "probe_${src}_s${st}_r$rep" 60 $P -mode recv -streams $st -total $((16<<30)) -send-cpu 2 -recv-cpu 1 -src $src
        cat "$O/probe_${src}_s${st}_r$rep.log" >> "$O/probe.jsonl"
      done
    done
  done
  step probe_anon_thp_splice_s8 60 $P -mode splice -streams 8 -total $((16<<30)) -send-cpu 2 -recv-cpu 1 -src anon_thp \
    -worker-cpus 3,4,5,6,7,129,130,131
  cat "$O/probe_anon_thp_splice_s8.log" >> "$O/probe.jsonl"
  ;;
splice)  # profiles/r3_splice: multiplexed-reader cost, recv() copy vs splice() into per-stream pipes
  { uname -r; cat /proc/sys/fs/pipe-max-size /proc/sys/fs/pipe-user-pages-soft; id -u;
    lscpu | grep -E "^(Model name|L3|NUMA node)"; } > "$O/env.txt" 2>&1
  P=custom_go_client_benchmark_amd/bin/splice_probe
  for rep in 1 2; do
    for st in 1 8; do
      for m in recv splice; do
        step "probe_${m}_s${st}_r$rep" 60 $P -mode $m -streams $st -total $((16<<30)) -send-cpu 2 -recv-cpu 1 \
          -worker-cpus 3,4,5,6,7,129,130,131
        cat "$O/probe_${m}_s${st}_r$rep.log" >> "$O/probe.jsonl"
      done
    done
  done
  step probe_splice_s8_2m 60 $P -mode splice -streams 8 -msg $((2<<20)) -total $((16<<30)) -send-cpu 2 -recv-cpu 1 \
    -worker-cpus 3,4,5,6,7,129,130,131
  step probe_splice_s48 60 $P -mode splice -streams 48 -total $((16<<30)) -send-cpu 2 -recv-cpu 1 \
    -worker-cpus 3,4,5,6,7,129,130,131,132,133,134,135
  step probe_recv_s48 60 $P -mode recv -streams 48 -total $((16<<30)) -send-cpu 2 -recv-cpu 1
  cat "$O"/probe_*_2m.log "$O"/probe_*_s48.log >> "$O/probe.jsonl"
  for rep in 1 2; do
    for v in 0 1; do
      step "bench_relay${v}_r$rep" 300 env GCSB_SPLICE_RECV=$v python3 bench.py --steps 20 --warmup 3 \
        --blocks list_read,ref_default --json-out "$O/bench_relay${v}_r$rep.json"
    done
  done
  ;;
stall)  # profiles/r3_sdma_engines: which hand-off HIP call blocks after a device sync
  step probe_default 200 python3 scripts/experiments/sync_stall_probe.py --reps 8
  step probe_hwq8 200 env GPU_MAX_HW_QUEUES=8 python3 scripts/experiments/sync_stall_probe.py --reps 8
  step probe_pool4 200 env GCSB_STREAMS=4 python3 scripts/experiments/sync_stall_probe.py --reps 8
  step bench 300 python3 bench.py --steps 20 --warmup 5
  step trace 300 rocprofv3 --hip-runtime-trace --memory-copy-trace --kernel-trace --output-format csv -d "$O/trace" \
    -o b -- python3 scripts/experiments/sync_stall_probe.py --reps 4 --variants sync
  ;;
engines)  # profiles/r3_sdma_engines: per-engine first-use cost; bench with the warm-up off / on
  step engines 120 env GCSB_WARM_ENGINES=0 python3 scripts/experiments/copy_engines_probe.py
  for i in 1 2; do
    for w in 0 1; do
      step "bench_w${w}_$i" 300 env GCSB_WARM_ENGINES=$w python3 bench.py --steps 20 --warmup 5 --list-objects 0
    done
  done
  ;;
write)  # profiles/r3_write: spliced vs copied send; endpoint CRC inline vs on a write worker
  for i in 1 2; do
    for v in "1 0 2" "1 1 2" "1 1 1" "0 0 2"; do
      set -- $v
      step "write_s$1_w$2_b$3_$i" 200 env GCSB_UPLOAD_SPLICE=$1 GCSB_SRV_WRITE_WORKER=$2 GCSB_SRV_WRITE_BUFS=$3 \
        python3 bench.py --workload write --steps 30 --warmup 3
    done
  done
  ;;
mux)  # profiles/r3_mux: ring geometry of the multiplexed list-read
  for i in 1 2; do
    for ring in 8x2MiB 2x1MiB 4x512KiB; do
      step "mux_${ring}_$i" 200 python3 bench.py --steps 5 --warmup 2 --side-steps 5 --blocks list_read,ref_default \
        --list-ring "$ring"
    done
  done
  ;;
b)  # profiles/r3_mux, r3_write: full bench, then the multiplexed and upload blocks twice
  step bench 300 python3 bench.py --steps 20 --warmup 5
  for i in 1 2; do
    step "mux_$i" 200 python3 bench.py --steps 5 --warmup 2 --side-steps 5 --blocks list_read,ref_default
    for w in 0 1; do
      step "write_w${w}_$i" 200 env GCSB_SRV_WRITE_WORKER=$w python3 bench.py --workload write --steps 30 --warmup 3
    done
  done
  ;;
check)  # profiles/r3_gpu_check, r3_rehearsal8: GPU suite, smoke, 8-rank gloo rehearsal, kernel profile
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step rehearsal8 500 env GCSB_DIST_BACKEND=gloo python3 bench.py --gpus 8 --object-size 64MiB --steps 5 --side-steps 3
  step rocprof 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof" -o bench -- \
    python3 bench.py --steps 10 --warmup 2
  ;;
benches)  # profiles/r3_gpu_check: three full benches back to back, host memory-management settings
  for i in 1 2 3; do
    step "bench_$i" 300 python3 bench.py --steps 20 --warmup 5
  done
  cat /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/enabled \
    /sys/kernel/mm/transparent_hugepage/defrag > "$O/host_mm.txt" 2>&1
  ;;
reader)  # profiles/r3_reader_cost: one gRPC stream's receive cost by component, then a bench
  step reader_cost 300 python3 scripts/experiments/reader_cost_probe.py --reps 3
  step bench 300 python3 bench.py --steps 20 --warmup 5
  grep -E "AnonHugePages|HugePages_|Hugepagesize" /proc/meminfo > "$O/meminfo.txt"
  ;;
bench_vs_probe)  # profiles/r3_reader_cost/session_f: bench (RCCL / gloo control plane) interleaved with the probe
  step bench_rccl_1 300 python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling
  step probe_1 200 python3 scripts/experiments/reader_cost_probe.py --reps 1
  step bench_gloo 300 env GCSB_DIST_BACKEND=gloo python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling
  step probe_2 200 python3 scripts/experiments/reader_cost_probe.py --reps 1
  step bench_rccl_2 300 python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling
  ;;
w48)  # profiles/r3_w48_tail: the 48-worker first-rep stall (thread states, syscalls, wait channels)
  step w48_default 200 python3 scripts/experiments/w48_tail_probe.py --reps 3
  step w48_warm20 200 python3 scripts/experiments/w48_tail_probe.py --reps 2 --warm-reads 20
  step w48_gap3 200 python3 scripts/experiments/w48_tail_probe.py --reps 2 --gap-s 3
  step w48_grpc 200 python3 scripts/experiments/w48_tail_probe.py --protocol grpc --reps 2 --slow-ms 30
  ;;
poll)  # profiles/r3_w48_tail/session_i: end-of-read event wait, runtime sync vs poll
  for k in 1 2; do
    step "list_sync_$k" 300 env GCSB_WAIT_POLL_US=0 python3 bench.py --steps 5 --warmup 2 --blocks list_read
    step "list_poll_$k" 300 env GCSB_WAIT_POLL_US=10 python3 bench.py --steps 5 --warmup 2 --blocks list_read
  done
  ;;
muxreader)  # profiles/r3_w48_tail/session_j: isolated reader core, list-read receive buffer
  step w48_http 200 python3 scripts/experiments/w48_tail_probe.py --reps 2
  for k in 1 2; do
    step "w48_grpc_shared_$k" 200 python3 scripts/experiments/w48_tail_probe.py --protocol grpc --reps 2 --sample-ms 0
    step "w48_grpc_isolate_$k" 200 python3 scripts/experiments/w48_tail_probe.py --protocol grpc --reps 2 --sample-ms 0 \
      --isolate-reader
    step "bench_shared_$k" 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read,ref_default --list-rcvbuf 0
    step "bench_isolate_$k" 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read,ref_default --list-rcvbuf 0 \
      --mux-reader isolate
    step "bench_rcvbuf_$k" 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read --list-rcvbuf 64MiB
  done
  ;;
wplace)  # profiles/r3_write/placement: config-5 upload, share vs pair placement, interleaved
  for k in 1 2 3; do
    for pl in share pair; do
      step "write_${pl}_$k" 200 python3 bench.py --workload write --steps 30 --warmup 3 --write-placement $pl
    done
  done
  ;;
spin)  # profiles/r3_w48_tail/spin: submitter polls for the next hand-off before it sleeps
  for k in 1 2 3; do
    step "spin0_$k" 300 env GCSB_SUBMIT_SPIN_US=0 python3 bench.py --steps 20 --warmup 5 --blocks list_read,sliced
    step "spin100_$k" 300 env GCSB_SUBMIT_SPIN_US=100 python3 bench.py --steps 20 --warmup 5 --blocks list_read,sliced
  done
  ;;
listiso)  # profiles/r3_w48_tail/listiso: config-3 list-read, reader core isolated vs shared (64 MiB rcvbuf both)
  for k in 1 2 3; do
    step "shared_$k" 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read
    step "isolate_$k" 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read --mux-reader isolate
  done
  ;;
recvdiag)  # profiles/r3_w48_tail/recvdiag: socket queue at every payload recv (GCSB_RECV_DIAG), headline + list-read
  for k in 1 2; do
    step "diag_$k" 300 env GCSB_RECV_DIAG=1 python3 bench.py --steps 20 --warmup 5 --blocks list_read,ref_default
  done
  ;;
align)  # profiles/r3_align: objects on page boundaries of the pattern (default) vs any byte (round 2)
  step probe 150 ./build/probes/align_probe
  for k in 1 2 3; do
    step "byte_$k" 300 env GCSB_PATTERN_ROT_ALIGN=1 python3 bench.py --steps 20 --warmup 5 \
      --blocks cpu_baseline,ceiling,list_read,ref_default
    step "page_$k" 300 python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling,list_read,ref_default
  done
  ;;
listring)  # profiles/r3_mux_thp/listring: list-read ring footprint (8 workers x ring), THP endpoint
  for k in 1 2 3; do
    for r in 8x2MiB 2x1MiB 4x1MiB; do
      step "r${r}_$k" 300 python3 bench.py --steps 20 --warmup 3 --blocks list_read --list-ring $r \
        --json-out "$O/r${r}_$k.json"
    done
  done
  ;;
final)  # profiles/r3_final: GPU suite, smoke, two full benches
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
  step bench_1 400 python3 bench.py
  step bench_2 400 python3 bench.py
  ;;
*)
  echo "unknown session $S" >&2
  exit 2
  ;;
esac
echo "session $S done"
