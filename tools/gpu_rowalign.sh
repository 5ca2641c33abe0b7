# Output row pitch A/B: 4-float (16 B) vs 32-float (128 B) granule, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rowalign; mkdir -p $OUT
for al in 4 32 4 32; do
  DSPCORE_ROW_ALIGN=$al timeout -k 10 300 python tools/tile_ab.py --tag "c5_al$al" --config c5 --channels 8192 2>&1 | grep -v amdgpu.ids | tee -a $OUT/timing.jsonl || exit 1
  DSPCORE_ROW_ALIGN=$al timeout -k 10 300 python tools/tile_ab.py --tag "c3_al$al" --channels 4096 32768 2>&1 | grep -v amdgpu.ids | tee -a $OUT/timing.jsonl || exit 1
done
python tools/tile_ab.py --compare c5_al4 c5_al32 | tee $OUT/compare.txt
