#!/bin/bash
# Evidence for bench.py's roofline object: kernel stats of one leg alone (LEG=dominant|t32),
# then one --pmc pass per counter group (FETCH_SIZE, WRITE_SIZE, SQ busy/LDS).
# Outputs under gpurun_out/roof_$LEG/.  Each GPU step is time-limited; stop at first failure.
LEG=${LEG:-dominant}
O=gpurun_out/roof_$LEG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o roof -- python tools/roofline_only.py $LEG > $O/stats.log 2>&1 || exit 1
tail -1 $O/stats.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o roof -- python tools/roofline_only.py $LEG > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o roof -- python tools/roofline_only.py $LEG > $O/write.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/sq -o roof -- python tools/roofline_only.py $LEG > $O/sq.log 2>&1 || exit 1

if [ "$LEG" = dominant ]; then
  python tools/roof_traffic.py $O $O/traffic.json "grouped weight gradients of the LF prior (16 Linears, 6400 tokens): wgrad_wide_kernel + wgrad_group_reduce_kernel" wgrad_wide_kernel wgrad_group_reduce_kernel
fi
if [ "$LEG" = wgrad ]; then
  python tools/roof_traffic.py $O $O/traffic.json "LF 64->64 3x3 conv weight+bias gradient over 6144 positions: conv_wgrad_w8_kernel + reduce_rows_kernel" conv_wgrad_w8_kernel reduce_rows_kernel
fi
if [ "$LEG" = rbbwd ]; then
  python tools/roof_traffic.py $O $O/traffic.json "fused ResBlock backward C=16 on (256,16,3,32): rb_bwd2_kernel + rb_bwd1_kernel + one batched ordered slab-sum launch" rb_bwd2_kernel rb_bwd1_kernel reduce_rows
fi
if [ "$LEG" = rb32bwd ]; then
  python tools/roof_traffic.py $O $O/traffic.json "fused ResBlock backward C=32 on (256,32,3,16): rb_bwd2_kernel + rb_bwd1_kernel (g / s planes) + conv_wgrad_w8_kernel<16,8> + the batched ordered slab sum" rb_bwd2_kernel rb_bwd1_kernel conv_wgrad_w8_kernel reduce_rows
fi
if [ "$LEG" = linfwd ]; then
  python tools/roof_traffic.py $O $O/traffic.json "LF prior Linear forward (6400x128)x(128x128) + bias + residual: gemm_rb2_kernel<64,true>" gemm_rb2_kernel
fi
if [ "$LEG" = vqassign ]; then
  python tools/roof_traffic.py $O $O/traffic.json "HF VQ codebook assignment, 24576 token rows x 512 codes x D 128 (straight-through, token-major copy): vq_assign_kernel" vq_assign_kernel
fi
if [ "$LEG" = t32 ]; then
  python tools/roof_traffic.py $O $O/traffic.json "HF ResBlock 128->128 3x3 conv on (256,128,3,32): conv_t32_kernel (pack-cached weights)" conv_t32_kernel
fi
if [ "$LEG" = attn ]; then
  python tools/roof_traffic.py $O $O/traffic.json "fused LF prior attention branch forward, 256 x 25 tokens: xattn_fwd_kernel" xattn_fwd_kernel
fi
if [ "$LEG" = n16 ]; then
  python tools/roof_traffic.py $O $O/traffic.json "HF 128->16 3x3 conv on (256,128,3,32): conv_n16_kernel" conv_n16_kernel
fi
if [ "$LEG" = rb64 ]; then
  python tools/roof_traffic.py $O $O/traffic.json "fused LF ResBlock(64,64) training forward on (256,64,3,8): w8_fwd1 + bn_stats_final + w8_fwd2" w8_fwd1_kernel bn_stats_final_kernel w8_fwd2_kernel
fi
echo roofline-done
