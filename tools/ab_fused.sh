set -e
for sh in 0 1 2 3; do
  echo "== shape $sh"; KS_TAG=_s$sh bash tools/kstats.sh lww_merge --option sets.fused_shape=$sh | grep -E "lww_fused|lww_split"
  echo "== shape $sh no look-back"; KS_TAG=_s${sh}d bash tools/kstats.sh lww_merge --option sets.fused_shape=$sh --option sets.fused_diag=1 | grep -E "lww_fused|lww_split"
done
