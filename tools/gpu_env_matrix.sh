#!/bin/bash
# Path-tracing kernel time (exp_timing.py, megakernel, child-pair walk) per workload under several
# environment settings, alternating rounds; optional parity subset first.
# usage: gpu_env_matrix.sh TAG "workloads" ROUNDS "ENV1" "ENV2" ...   (ENV = space-separated K=V, or "-")
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; WLS=$2; ROUNDS=$3; shift 3
mkdir -p gpurun_out
OUT=gpurun_out/envmx_$TAG.log
: > $OUT
for r in $(seq $ROUNDS); do
  for cfg in "$@"; do
    for w in $WLS; do
      envs=""; [ "$cfg" != "-" ] && envs="$cfg"
      res=$(env $envs timeout -k 10 120 python tools/exp_timing.py --workload $w --frames 30 --backends megakernel --layouts pairs --no-mesh-variant 2>&1 | tail -1) || { echo "FAIL $cfg $w: $res" >> $OUT; exit 1; }
      echo "r$r [$cfg] $w $res" >> $OUT
    done
  done
done
