// scan.hip -- device-wide exclusive scan (uint32 counts -> uint64 offsets).
// Used by RefMerge (tiles per replica, inclusion counts of large batches) and
// the gossip assembly: scan_lb (scan.hpp), reduce / scan the tile sums /
// apply, with no cross-workgroup waiting.
#include "scan.hpp"

namespace crdt {

size_t scan_tmp_bytes(size_t n) { return scan_lb_tmp_bytes(n); }

int exclusive_scan_u32(crdt_ctx *ctx, const uint32_t *in, uint64_t *out, size_t n, void *tmp) {
    return scan_lb(ctx, CountSrc{in}, NoAct{}, n, 0, out, tmp);
}

}  // namespace crdt
