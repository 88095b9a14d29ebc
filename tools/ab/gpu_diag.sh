#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/aten_ops.py > gpurun_out/aten_ops.log 2>&1
rc=$?; head -5 gpurun_out/aten_ops.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_shapes_bench.py > gpurun_out/conv_shapes.log 2>&1
rc=$?; cat gpurun_out/conv_shapes.log; exit $rc
