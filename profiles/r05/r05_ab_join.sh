#!/bin/bash
# Round 5: p1v with the own column's loads joined to the first cluster round trip (OPT 512: b1v
# and the self bound behind the ring; exact, max/min commute) against the product build.
#   (r05o) lib_x512: that form as compiled (66 VGPRs, 7 waves/SIMD); lib_x512w8: held to 8 waves
#   (64 VGPRs + 6 spilled).  The ring loop's header still waited for the own loads (a zero write
#   into a pending load's registers), so r05p peels the first ring batch (OPT 4096): its loads go
#   out ahead of the own column's and one wait covers both --
#   lib_x4608: 512 | 4096 (66 VGPRs, 7 waves); lib_x6656: + unconditional gathers (2048).
#   r05q: lib_x25088 = 512 | 8192 | 16384 at 64 VGPRs / 8 waves: unconditional ring gathers with a
#   drain at the ring loop's latch (no header wait: LO/ttf ride the first ring trip), fct_adf_v
#   loaded in the first edge batch's trip (6 dependent trips instead of 7)
# Full-size exact checks first (1 and 6 tracers), then interleaved A/B.
# MEASURED AND REVERTED (profiles/INDEX_r05.md): every variant exact; the best, x25088 at 8 waves,
# p1v -0.2..-0.5 % -- within noise.  The kernel variants (p1_body OPT bits 512..16384, edge_batch,
# the F2A_P1V_EXTRA hook) are not in the tree any more; this script documents how they were run.
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate.so
for v in ${VARIANTS:-x25088}; do
    FESOM2_LIB_DIR=fesom2-accelerate_amd/lib_$v timeout -k 10 300 python bench.py --no-cpu-baseline --extras none \
        > gpurun_out/${TAG:-r05q}_${v}_1tr_check.json 2> gpurun_out/${TAG:-r05q}_${v}_1tr_check.err
    FESOM2_LIB_DIR=fesom2-accelerate_amd/lib_$v timeout -k 10 300 python bench.py --no-cpu-baseline --extras none --tracers 6 \
        > gpurun_out/${TAG:-r05q}_${v}_6tr_check.json 2> gpurun_out/${TAG:-r05q}_${v}_6tr_check.err
done
echo "checks done"
A="FESOM2_LIB_DIR=fesom2-accelerate_amd/lib"
B="FESOM2_LIB_DIR=fesom2-accelerate_amd/lib_${VARIANTS:-x25088}"
ROUNDS=5 STEPS=40 timeout -k 10 600 bash tools/sweep_env.sh "$A" "$B"
cp gpurun_out/sweep.txt gpurun_out/${TAG:-r05q}_sweep_join_1tr.txt
ROUNDS=4 STEPS=20 BENCH_ARGS="--tracers 6" timeout -k 10 600 bash tools/sweep_env.sh "$A" "$B"
cp gpurun_out/sweep.txt gpurun_out/${TAG:-r05q}_sweep_join_6tr.txt
echo "sweeps done"
