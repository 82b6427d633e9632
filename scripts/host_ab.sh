#!/bin/bash
# Host-engine A/B on the GPU box (item 2 of the round-6 verdict): prebuilt variants of bench/bench_tcp_server under
# scratch_ab/, run in alternation -- the CPU twin's dispatch alone (twin_timed) and the best GPU leg beside the
# reference's own server (resident_pair) -- N rounds.   bash scripts/host_ab.sh <tag> <rounds> <binary>...
set -o pipefail
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq $N); do
  for b in "$@"; do
    timeout -k 5 60 $b 256 3000 twin_timed > $OUT/$(basename $b).twin.$r.json 2>/dev/null || { echo "$b twin rc=$?"; exit 1; }
    timeout -k 5 90 $b 256 1000 resident_pair > $OUT/$(basename $b).pair.$r.json 2>/dev/null || { echo "$b pair rc=$?"; exit 1; }
  done
done
python3 - "$OUT" "$@" <<'P'
import json, sys, glob, os, statistics
out, bins = sys.argv[1], sys.argv[2:]
for b in bins:
    n = os.path.basename(b)
    tw = [json.load(open(f))["cpu_rxbatch_512_pipelined_release_path_timed"] for f in sorted(glob.glob(f"{out}/{n}.twin.*.json"))]
    pr = [json.load(open(f)) for f in sorted(glob.glob(f"{out}/{n}.pair.*.json"))]
    d = [x["ns_per_frame_dispatch"] for x in tw]
    g = [x["gpu_rxbatch_512_pipelined_resident_release_path"]["mframes_per_s"] for x in pr]
    rf = [x["reference_server_release_build"]["mframes_per_s"] for x in pr]
    print(f"{n:14s} dispatch ns min {min(d):6.2f} med {statistics.median(d):6.2f} | gpu leg Mfps med {statistics.median(g):6.2f} "
          f"| reference med {statistics.median(rf):6.2f} | ratio med {statistics.median([a / b for a, b in zip(g, rf)]):.3f}")
P
