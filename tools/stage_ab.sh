set -o pipefail
for r in a b; do for w in lww_merge orset_merge; do for k in 1 9; do
  bash tools/kstats.sh st$w$k$r $w --option sets.knobs=$k | grep -E "k_lww_write|k_or_write" | sed "s/^/$w k$k /"
done; done; done
