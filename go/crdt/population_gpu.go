//go:build cgo && rocm

// Device-level entry points for hosts whose replica state already lives in
// HBM (populations, sharded state), over the same C-ABI (include/crdt_amd.h).
// Uncompiled in the build image (no Go toolchain).
package crdt

/*
#include <stdlib.h>
#include "crdt_amd.h"
*/
import "C"

import (
	"bytes"
	"fmt"
	"log"
	"unsafe"
)

// GossipTick: one gossip tick for the replicas this process hosts
// (main.go:226-258).  Each binary pull is parked at ingest (validated on the
// host, its upload to HBM started); every ingested server merges in ONE
// batched device call.
func GossipTick(servers []*Server, bodies [][]byte) {
	hs := make([]*C.crdt_server, 0, len(servers))
	for i, s := range servers {
		if len(bodies[i]) == 0 {
			continue // a failed GET: no merge this round (main.go:234-239)
		}
		var out C.int
		C.crdt_server_ingest_binary(s.gpu, (*C.char)(unsafe.Pointer(&bodies[i][0])), C.size_t(len(bodies[i])), &out)
		if out == 0 {
			hs = append(hs, s.gpu)
		}
	}
	if len(hs) == 0 {
		return
	}
	if err := status(C.crdt_servers_merge(&hs[0], C.size_t(len(hs)))); err != nil {
		log.Printf("batched merge skipped, every server unchanged: %v", err) // (the next tick retries)
		return
	}
	for _, s := range servers {
		s.CurrentState = s.currentState()
	}
}

// GCounterJoin: a G-Counter population join on device pointers (crdt_dev_alloc).
func GCounterJoin(aDev, bDev, outDev unsafe.Pointer, rows, nodes int) error {
	return status(C.crdt_gcounter_join(gpuCtx, (*C.uint64_t)(aDev), (*C.uint64_t)(bDev), (*C.uint64_t)(outDev),
		C.size_t(rows), C.size_t(nodes)))
}

// UniqueID: rank 0 makes the RCCL id and ships it to the other ranks.
func UniqueID() ([]byte, error) {
	id := make([]byte, C.CRDT_SHARD_ID_BYTES)
	return id, status(C.crdt_shard_unique_id(unsafe.Pointer(&id[0]), C.size_t(len(id))))
}

// JoinPopulation: one process per GPU (the shape of bench.py --gpus N); each
// rank folds its row shard and one call all-reduces the folds over RCCL
// (ncclAllReduce(ncclUint64, ncclMax)): outDev = the global join.
func JoinPopulation(id []byte, nranks, rank int, shard unsafe.Pointer, rows, nodes int, outDev unsafe.Pointer) error {
	var comm *C.crdt_comm
	if err := status(C.crdt_shard_comm_init_rank(gpuCtx, unsafe.Pointer(&id[0]), C.int(nranks), C.int(rank), &comm)); err != nil {
		return err
	}
	defer C.crdt_shard_comm_destroy(comm)
	sh := []*C.uint64_t{(*C.uint64_t)(shard)}
	nr := []C.size_t{C.size_t(rows)}
	out := []*C.uint64_t{(*C.uint64_t)(outDev)}
	if err := status(C.crdt_shard_fold_max_u64(comm, &sh[0], &nr[0], C.size_t(nodes), &out[0])); err != nil {
		return err
	}
	return status(C.crdt_shard_sync(comm))
}

// MergeShardedBatch: merge() of one batch of replicas whose logs are split by
// ts range over the ranks -- the whole protocol (global max(L), local merge,
// accumulator all-reduces, finalize) on the communicator's stream.
func MergeShardedBatch(comm *C.crdt_comm, in *C.crdt_refmerge_in, out *C.crdt_refmerge_out) error {
	if err := status(C.crdt_shard_refmerge(comm, in, out)); err != nil {
		return err
	}
	return status(C.crdt_shard_sync(comm))
}

// GossipRound: the gossip loop of main.go:226-261 for all the replicas this
// rank hosts; every rank passes the same draw (friend ids, -1 = a dead
// friend, main.go:230, :234-239).  One call moves exactly the pulled Diffs
// over xGMI and merges.
func GossipRound(comm *C.crdt_comm, pop *C.crdt_population, draw []int64) error {
	pops := []*C.crdt_population{pop}
	return status(C.crdt_population_round_sharded(comm, &pops[0], (*C.int64_t)(unsafe.Pointer(&draw[0])),
		C.uint64_t(len(draw))))
}

func uploadBytes(b []byte) (unsafe.Pointer, error) {
	var dev unsafe.Pointer
	if err := status(C.crdt_dev_alloc(gpuCtx, C.size_t(len(b)), &dev)); err != nil || len(b) == 0 {
		return dev, err
	}
	if err := status(C.crdt_memcpy_h2d(gpuCtx, dev, unsafe.Pointer(&b[0]), C.size_t(len(b)))); err != nil {
		C.crdt_dev_free(gpuCtx, dev)
		return nil, err
	}
	return dev, nil
}

// GossipRoundWire: the same loop when the Diffs come over HTTP
// (main.go:231-256): bodies[i] is replica i's GET body (nil after a failed
// request), decoded and merged on the device; keys / vals are the context's
// string tables (vals seeded with the population's strings at their ids).
func GossipRoundWire(pop *C.crdt_population, keys, vals *C.crdt_strtab, bodies [][]byte) error {
	off := make([]uint64, len(bodies)+1)
	for i, b := range bodies {
		off[i+1] = off[i] + uint64(len(b))
	}
	dev, err := uploadBytes(bytes.Join(bodies, nil))
	if err != nil {
		return err
	}
	defer C.crdt_dev_free(gpuCtx, dev)
	st := make([]uint32, len(bodies))
	if rc := C.crdt_population_round_wire(pop, keys, vals, (*C.uint8_t)(dev), (*C.uint64_t)(unsafe.Pointer(&off[0])),
		(*C.uint32_t)(unsafe.Pointer(&st[0]))); rc != C.CRDT_OK {
		return fmt.Errorf("wire round refused (body status %v): %w", st, status(rc)) // decode those on the host
	}
	return nil
}

// MergeDistributedLWW: keyed sets of a distributed population -- this rank's
// own sorted LWW tuples (a, b); with gather every rank ends with the whole
// merged state in out.
func MergeDistributedLWW(comm *C.crdt_comm, a, b *C.crdt_tuples, na, nb int, out *C.crdt_tuples, capacity int) (int, error) {
	cna, cnb := []C.size_t{C.size_t(na)}, []C.size_t{C.size_t(nb)}
	n := []C.size_t{0}
	err := status(C.crdt_shard_lww_merge_local(comm, a, &cna[0], b, &cnb[0], out, C.size_t(capacity), &n[0], 1))
	return int(n[0]), err
}

// D2Merger: unsorted (D2) set state merged every round with no host
// synchronisation -- plan once per shape, then enqueue (also capturable in a
// HIP graph).  A call whose inputs leave the plan writes count = 2^64 - 1 and
// raises CRDT_DEV_PLAN: re-plan and run the unplanned call for that round.
type D2Merger struct {
	plan   C.crdt_set_plan
	na, nb C.size_t
}

func NewD2Merger(a, b *C.crdt_tuples, na, nb int) (*D2Merger, error) {
	m := &D2Merger{na: C.size_t(na), nb: C.size_t(nb)}
	// mode 0 = LWW; widen 1: field ranges padded by 1/256 of their span for drift
	err := status(C.crdt_set_merge_plan(gpuCtx, 0, a, m.na, b, m.nb, 1, &m.plan))
	return m, err
}

func (m *D2Merger) Enqueue(a, b, out *C.crdt_tuples, countDev *C.uint64_t) error {
	return status(C.crdt_lww_merge_unsorted_planned(gpuCtx, &m.plan, a, m.na, b, m.nb, out, countDev))
}

// RCCLInfo: which RCCL the process runs (for the service's logs / metrics).
func RCCLInfo() (int, string) {
	var v C.int
	buf := make([]byte, 512)
	if status(C.crdt_rccl_info(&v, (*C.char)(unsafe.Pointer(&buf[0])), 512)) != nil {
		return 0, ""
	}
	return int(v), C.GoString((*C.char)(unsafe.Pointer(&buf[0])))
}
