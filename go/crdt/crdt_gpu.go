//go:build cgo && rocm

// Package crdt is the Go side of the drop-in boundary: the reference's Server
// (main.go:23-33), NewServer (main.go:102-113) and merge() (main.go:35-100),
// with the state held by libcrdt_amd (include/crdt_amd.h) and every merge run
// on the GPU.  In the reference repo, change the package line to main and
// delete main.go:23-113: every call site (main.go:159, :187, :255, :257)
// compiles unchanged.  Uncompiled in the build image (no Go toolchain).
package crdt

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../crdt_amd -lcrdt_amd -Wl,-rpath,${SRCDIR}/../../crdt_amd
#include <stdlib.h>
#include "crdt_amd.h"
*/
import "C"

import (
	"fmt"
	"log"
	"sync"
	"unsafe"
)

// Data and Command as main.go:19-21 declares them.
type Data map[string]string
type Command map[string]string

var gpuCtx *C.crdt_ctx // one context per process/GPU (NULL stream = the device's default stream)

func init() {
	if rc := C.crdt_ctx_create(0, nil, &gpuCtx); rc != C.CRDT_OK {
		log.Fatalf("crdt_amd: %s", C.GoString(C.crdt_status_str(rc))) // no GPU: the process cannot serve
	}
}

func status(rc C.int) error {
	if rc == C.CRDT_OK {
		return nil
	}
	return fmt.Errorf("crdt_amd: %s (%d)", C.GoString(C.crdt_status_str(rc)), int(rc))
}

// gpuLog stands in for the gods treemap of main.go:26-27: the method names
// the reference calls, the storage on the C side (HBM-resident between merges).
type gpuLog struct {
	srv    *C.crdt_server
	remote bool
}

// Server keeps the reference's fields (main.go:23-33).
type Server struct {
	InitialState Data
	CurrentState Data
	Diff         *gpuLog
	RemoteDiff   *gpuLog
	Port         int
	LastReceived int64
	FriendList   []string
	Alive        bool
	Lock         sync.Mutex
	gpu          *C.crdt_server
}

// kv marshals a Go map into the parallel (ptr, len) arrays of the C-ABI.
// The C side copies everything before returning (no Go pointer is retained).
func kv(m map[string]string) (**C.char, *C.size_t, **C.char, *C.size_t, C.size_t, func()) {
	n := len(m)
	if n == 0 {
		return nil, nil, nil, nil, 0, func() {}
	}
	ks := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	vs := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	kl := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0))))
	vl := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0))))
	kp := (*[1 << 28]*C.char)(ks)[:n:n]
	vp := (*[1 << 28]*C.char)(vs)[:n:n]
	klp := (*[1 << 28]C.size_t)(kl)[:n:n]
	vlp := (*[1 << 28]C.size_t)(vl)[:n:n]
	i := 0
	for k, v := range m {
		kp[i], klp[i] = C.CString(k), C.size_t(len(k))
		vp[i], vlp[i] = C.CString(v), C.size_t(len(v))
		i++
	}
	free := func() {
		for j := 0; j < n; j++ {
			C.free(unsafe.Pointer(kp[j]))
			C.free(unsafe.Pointer(vp[j]))
		}
		C.free(ks)
		C.free(vs)
		C.free(kl)
		C.free(vl)
	}
	return (**C.char)(ks), (*C.size_t)(kl), (**C.char)(vs), (*C.size_t)(vl), C.size_t(n), free
}

// NewServer(port, initialState, friendList) (main.go:102-113).
func NewServer(port int, initialState Data, friendList []string) *Server {
	s := &Server{InitialState: initialState, Port: port, FriendList: friendList, Alive: true}
	if rc := C.crdt_server_new(gpuCtx, C.int(port), &s.gpu); rc != C.CRDT_OK {
		log.Fatalf("NewServer: %v", status(rc))
	}
	k, kl, v, vl, n, free := kv(initialState)
	defer free()
	if rc := C.crdt_server_init_state(s.gpu, k, kl, v, vl, n); rc != C.CRDT_OK {
		log.Fatalf("NewServer: %v", status(rc))
	}
	s.Diff, s.RemoteDiff = &gpuLog{s.gpu, false}, &gpuLog{s.gpu, true}
	s.CurrentState = initialState // main.go:104-105: the same map
	return s
}

// Close releases the C-side state (the reference's servers live forever).
func (server *Server) Close() error {
	err := status(C.crdt_server_free(server.gpu))
	server.gpu = nil
	return err
}

// Put: Diff.Put(ts, &data) stores a *Command (main.go:187); any other value
// is a remote map (main.go:68, :255).
func (l *gpuLog) Put(key interface{}, value interface{}) {
	ts := key.(int64) // utils.Int64Comparator would panic on anything else (main.go:106)
	var m map[string]string
	local := 0
	switch v := value.(type) {
	case *Command:
		m, local = map[string]string(*v), 1
	case map[string]string:
		m = v
	}
	k, kl, vv, vl, n, free := kv(m)
	defer free()
	var rc C.int
	if l.remote {
		rc = C.crdt_server_remote_put(l.srv, C.int64_t(ts), k, kl, vv, vl, n)
	} else {
		rc = C.crdt_server_diff_put(l.srv, C.int64_t(ts), C.int(local), k, kl, vv, vl, n)
	}
	if rc != C.CRDT_OK {
		log.Printf("Put(%d): %v", ts, status(rc))
	}
}

// Keys: ascending timestamps (treemap Keys under Int64Comparator, main.go:45-48).
func (l *gpuLog) Keys() []interface{} {
	var n C.size_t
	if l.remote {
		C.crdt_server_remote_len(l.srv, &n)
	} else {
		C.crdt_server_diff_len(l.srv, &n)
	}
	if n == 0 {
		return nil
	}
	ts := make([]C.int64_t, int(n))
	if l.remote {
		C.crdt_server_remote_keys(l.srv, &ts[0], n, &n)
	} else {
		C.crdt_server_diff_keys(l.srv, &ts[0], nil, n, &n)
	}
	out := make([]interface{}, int(n))
	for i := range out {
		out[i] = int64(ts[i])
	}
	return out
}

// ToJSON: the Gossip handler's body (main.go:159).
func (l *gpuLog) ToJSON() ([]byte, error) {
	var n C.size_t
	var st C.int
	C.crdt_server_gossip_json(l.srv, nil, 0, &n, &st) // CRDT_E_RANGE: n = the size needed
	buf := make([]byte, int(n)+1)
	if rc := C.crdt_server_gossip_json(l.srv, (*C.char)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)), &n, &st); rc != C.CRDT_OK {
		return nil, status(rc)
	}
	return buf[:int(n)], nil
}

// Merge is merge() with its status: nil, or the device error after which
// Diff, RemoteDiff and CurrentState are exactly as they were.
func (server *Server) Merge() error {
	server.Alive = false // main.go:41
	server.Lock.Lock()   // main.go:43-44
	defer server.Lock.Unlock()
	defer func() { server.Alive = true }() // main.go:99, also after a failed merge
	if err := status(C.crdt_server_merge(server.gpu)); err != nil {
		return err
	}
	server.CurrentState = server.currentState() // main.go:76: rebuilt from empty
	return nil
}

// merge replaces (*Server).merge() (main.go:35-100): the same effect on Diff,
// RemoteDiff and CurrentState, bit for bit, computed on the GPU.  Like the
// reference it never fails: a device error leaves the state untouched and the
// pull in RemoteDiff for the next round (no CPU fallback).
func (server *Server) merge() {
	if err := server.Merge(); err != nil {
		log.Printf("merge on :%d skipped, state unchanged: %v", server.Port, err)
	}
}

// currentState: CurrentState as the C side holds it (GetState, main.go:129-139).
func (server *Server) currentState() Data {
	var n C.size_t
	C.crdt_server_state_len(server.gpu, &n)
	out := make(Data, int(n))
	for i := C.size_t(0); i < n; i++ {
		var k, v *C.char
		var kl, vl C.size_t
		C.crdt_server_state_at(server.gpu, i, &k, &kl, &v, &vl)
		out[C.GoStringN(k, C.int(kl))] = C.GoStringN(v, C.int(vl))
	}
	return out
}

// Ingest decodes a gossip pull (main.go:245-256) in one call: 0 = ingested
// (merge next), 1 = skip the round, 2 = the reference's goroutine returns.
func (server *Server) Ingest(body []byte) int {
	var out C.int
	if len(body) == 0 {
		C.crdt_server_ingest_json(server.gpu, nil, 0, &out)
	} else {
		C.crdt_server_ingest_json(server.gpu, (*C.char)(unsafe.Pointer(&body[0])), C.size_t(len(body)), &out)
	}
	return int(out)
}

// AddCommand body after the JSON decode (main.go:187-209): the HTTP status;
// the Go CurrentState follows the C side.
func (server *Server) AddCommand(tsMs int64, data Command) int {
	k, kl, v, vl, n, free := kv(data)
	defer free()
	var st C.int
	C.crdt_server_add_command(server.gpu, C.int64_t(tsMs), k, kl, v, vl, n, &st)
	server.CurrentState = server.currentState()
	return int(st)
}
