#!/bin/bash
# One compile-time variant (build_variants/NAME/libpt.so): the walk's bit-exact GPU tests through
# it, then a whole-frame A/B against the in-tree build. usage: gpu_variant_check.sh NAME "workloads" [-k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
NAME=$1; WLS=${2:-"dragon bunny helmet"}; K=${3:-"bitexact and (bunny or dragon or helmet or stream)"}
PT_LIBPT=$PWD/build_variants/$NAME/libpt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > gpurun_out/variant_${NAME}_pytest.log 2>&1 || exit $?
tools/gpu_frame_ab.sh $NAME "$WLS"
