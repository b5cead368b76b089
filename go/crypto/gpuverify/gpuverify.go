// Package gpuverify batches tendermint secp256k1 VerifyBytes onto AMD MI355X
// GPUs through libgpuverify (include/gpuverify.h).
//
// It replaces, for a whole batch at once, the per-signature call
//
//	x/auth/ante/sigverify.go:210   pubKey.VerifyBytes(signBytes, sig)
//
// with identical results: ok[i] == pubs[i].VerifyBytes(msgs[i], sigs[i]).
// Every infrastructure failure (no device, HIP error, allocation failure,
// a key that could not be cached) sends the affected leaves to the reference
// VerifyBytes on the CPU, so a device problem can slow a node down but never
// change a verdict (fail closed, SURVEY.md §5).
//
// Source-level only in this repository: the build image has no Go toolchain.
// The same C ABI is exercised by the repository's C++/Python tests.
package gpuverify

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../cosmos-sdk-rootchain_amd/lib -lgpuverify -Wl,-rpath,${SRCDIR}/../../../cosmos-sdk-rootchain_amd/lib
#include <stdlib.h>
#include <stdint.h>
#include "gpuverify.h"
*/
import "C"

import (
	"errors"
	"sync"
	"unsafe"

	"github.com/tendermint/tendermint/crypto/ed25519"
	"github.com/tendermint/tendermint/crypto/secp256k1"
)

// maxBatchBytes bounds one library call's staging buffers (the array-cast
// idiom below needs a fixed upper bound; larger batches are split).
const maxBatchBytes = 1 << 30

// Verifier verifies a batch of secp256k1 leaves:
// ok[i] == pubs[i].VerifyBytes(msgs[i], sigs[i]).
type Verifier interface {
	VerifyBatch(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool
}

// EdVerifier verifies a batch of ed25519 leaves (multisig sub-keys):
// ok[i] == pubs[i].VerifyBytes(msgs[i], sigs[i]).
type EdVerifier interface {
	VerifyBatchEd25519(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool
}

// CPU is the reference path, one VerifyBytes per leaf (tendermint
// secp256k1_nocgo.go, ed25519.go).  It is the fallback of GPU and a Verifier
// of its own.
type CPU struct{}

// VerifyBatchEd25519 implements EdVerifier.
func (CPU) VerifyBatchEd25519(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool {
	ok := make([]bool, len(pubs))
	for i := range pubs {
		ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i])
	}
	return ok
}

// VerifyBatch implements Verifier.
func (CPU) VerifyBatch(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
	ok := make([]bool, len(pubs))
	for i := range pubs {
		ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i])
	}
	return ok
}

// GPU is a libgpuverify context on one or more HIP devices.  Safe for
// concurrent use: the library serialises calls per device, and the key-cache
// maps below are guarded by mu.
type GPU struct {
	ctx       *C.gv_ctx
	closeOnce sync.Once

	// CPUBelow routes batches smaller than this to the CPU (VerifyBatchRouted):
	// below the measured crossover a VerifyBytes loop answers first (one core:
	// ~0.21 ms per signature; the sliced small-batch kernels: ~0.26 ms for up
	// to 1,024 signatures, DESIGN.md §6.3).
	CPUBelow int

	mu      sync.Mutex
	slots   map[secp256k1.PubKeySecp256k1]uint32 // key -> key-arena slot (gv_keys_load)
	slotGen uint64                               // gv_keys_generation the slot map belongs to
}

var (
	_ Verifier   = (*GPU)(nil)
	_ EdVerifier = (*GPU)(nil)
	_ EdVerifier = CPU{}
)

// Open binds the listed HIP devices (nil or empty = every visible device).
func Open(devices []int) (*GPU, error) {
	var ids *C.int
	if len(devices) > 0 {
		// Go ints are 64-bit: copy into a C int array (cgo: no Go pointers kept)
		cids := (*C.int)(C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(C.int(0)))))
		defer C.free(unsafe.Pointer(cids))
		arr := (*[1 << 16]C.int)(unsafe.Pointer(cids))[:len(devices):len(devices)]
		for i, d := range devices {
			arr[i] = C.int(d)
		}
		ids = cids
	}
	var ctx *C.gv_ctx
	if rc := C.gv_open(ids, C.int(len(devices)), &ctx); rc != 0 {
		return nil, errors.New("gpuverify: gv_open: " + C.GoString(C.gv_strerror(rc)))
	}
	return &GPU{ctx: ctx, CPUBelow: 4, slots: map[secp256k1.PubKeySecp256k1]uint32{}}, nil
}

// Close releases the context (idempotent).
func (g *GPU) Close() { g.closeOnce.Do(func() { C.gv_close(g.ctx) }) }

// SetOption forwards to gv_set_option ("max_batch", "lat_max", "pipe_chunk", ...).
func (g *GPU) SetOption(key string, val int64) error {
	ck := C.CString(key)
	defer C.free(unsafe.Pointer(ck))
	if rc := C.gv_set_option(g.ctx, ck, C.longlong(val)); rc != 0 {
		return errors.New("gpuverify: gv_set_option(" + key + "): " + C.GoString(C.gv_strerror(rc)))
	}
	return nil
}

// cbuf is a C allocation viewed as a Go byte slice (freed by free()).
type cbuf struct {
	p unsafe.Pointer
	b []byte
}

func newCBuf(n int) cbuf {
	if n < 1 {
		n = 1
	}
	p := C.malloc(C.size_t(n))
	return cbuf{p, (*[maxBatchBytes]byte)(p)[:n:n]}
}
func (c cbuf) free() { C.free(c.p) }

// VerifyBatch implements Verifier.  Leaves whose signature is not 64 bytes
// are false without reaching the GPU (VerifyBytes' first check).  On any
// nonzero return the whole call is re-verified on the CPU.
func (g *GPU) VerifyBatch(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
	n := len(pubs)
	ok := make([]bool, n)
	idx := make([]int, 0, n)
	total := 0
	for i := range pubs {
		if len(sigs[i]) == 64 {
			idx = append(idx, i)
			total += len(msgs[i])
		}
	}
	if len(idx) == 0 {
		return ok
	}
	if total+97*len(idx) > maxBatchBytes { // split oversize batches
		h := len(pubs) / 2
		copy(ok, g.VerifyBatch(pubs[:h], msgs[:h], sigs[:h]))
		copy(ok[h:], g.VerifyBatch(pubs[h:], msgs[h:], sigs[h:]))
		return ok
	}
	m := len(idx)
	pub, sig, blob, off, ln, out := newCBuf(33*m), newCBuf(64*m), newCBuf(total), newCBuf(8*m), newCBuf(4*m), newCBuf(m)
	defer func() { pub.free(); sig.free(); blob.free(); off.free(); ln.free(); out.free() }()
	o := (*[maxBatchBytes / 8]uint64)(off.p)[:m:m]
	l := (*[maxBatchBytes / 4]uint32)(ln.p)[:m:m]
	pos := 0
	for k, i := range idx {
		copy(pub.b[33*k:], pubs[i][:])
		copy(sig.b[64*k:], sigs[i])
		o[k], l[k] = uint64(pos), uint32(len(msgs[i]))
		pos += copy(blob.b[pos:], msgs[i])
	}
	rc := C.gv_verify_msgs(g.ctx, C.size_t(m), (*C.uint8_t)(pub.p), (*C.uint8_t)(sig.p), (*C.uint8_t)(blob.p),
		(*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
	for k, i := range idx {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
		}
	}
	return ok
}

// VerifyBatchEd25519 implements EdVerifier with gv_verify_ed25519_msgs (go1.14
// crypto/ed25519 semantics on the GPU).  Same fail-closed rule as VerifyBatch.
func (g *GPU) VerifyBatchEd25519(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool {
	n := len(pubs)
	ok := make([]bool, n)
	idx := make([]int, 0, n)
	total := 0
	for i := range pubs {
		if len(sigs[i]) == 64 { // VerifyBytes: len(sig) != SignatureSize -> false
			idx = append(idx, i)
			total += len(msgs[i])
		}
	}
	if len(idx) == 0 {
		return ok
	}
	if total+108*len(idx) > maxBatchBytes {
		h := len(pubs) / 2
		copy(ok, g.VerifyBatchEd25519(pubs[:h], msgs[:h], sigs[:h]))
		copy(ok[h:], g.VerifyBatchEd25519(pubs[h:], msgs[h:], sigs[h:]))
		return ok
	}
	m := len(idx)
	pub, sig, blob, off, ln, out := newCBuf(32*m), newCBuf(64*m), newCBuf(total), newCBuf(8*m), newCBuf(4*m), newCBuf(m)
	defer func() { pub.free(); sig.free(); blob.free(); off.free(); ln.free(); out.free() }()
	o := (*[maxBatchBytes / 8]uint64)(off.p)[:m:m]
	l := (*[maxBatchBytes / 4]uint32)(ln.p)[:m:m]
	pos := 0
	for k, i := range idx {
		copy(pub.b[32*k:], pubs[i][:])
		copy(sig.b[64*k:], sigs[i])
		o[k], l[k] = uint64(pos), uint32(len(msgs[i]))
		pos += copy(blob.b[pos:], msgs[i])
	}
	rc := C.gv_verify_ed25519_msgs(g.ctx, C.size_t(m), (*C.uint8_t)(pub.p), (*C.uint8_t)(sig.p), (*C.uint8_t)(blob.p),
		(*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
	for k, i := range idx {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
		}
	}
	return ok
}

// VerifyBatchRouted sends batches below CPUBelow to the CPU (where a
// VerifyBytes loop answers before a GPU round trip) and the rest to the GPU.
func (g *GPU) VerifyBatchRouted(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
	if len(pubs) < g.CPUBelow {
		return CPU{}.VerifyBatch(pubs, msgs, sigs)
	}
	return g.VerifyBatch(pubs, msgs, sigs)
}

// ---- account key cache (gv_keys_load, SURVEY.md §8f-2)

// slotsFor returns each key's arena slot, loading the keys not yet cached
// with ONE gv_keys_load call.  loaded[i] is false when key i could not be
// cached (the load failed): the caller verifies that leaf on the CPU --
// never a sentinel slot, whose keyed verify would read as a rejection.
func (g *GPU) slotsFor(pubs []secp256k1.PubKeySecp256k1) (slots []uint32, loaded []bool) {
	g.mu.Lock()
	defer g.mu.Unlock()
	if gen := uint64(C.gv_keys_generation(g.ctx)); gen != g.slotGen {
		// the arena was reset elsewhere: every cached slot may name another key now
		g.slots = map[secp256k1.PubKeySecp256k1]uint32{}
		g.slotGen = gen
	}
	slots = make([]uint32, len(pubs))
	loaded = make([]bool, len(pubs))
	var fresh []secp256k1.PubKeySecp256k1
	seen := map[secp256k1.PubKeySecp256k1]bool{}
	for i, p := range pubs {
		if s, ok := g.slots[p]; ok {
			slots[i], loaded[i] = s, true
		} else if !seen[p] {
			seen[p] = true
			fresh = append(fresh, p)
		}
	}
	if len(fresh) > 0 {
		buf := newCBuf(33 * len(fresh))
		out := newCBuf(4 * len(fresh))
		defer func() { buf.free(); out.free() }()
		for k, p := range fresh {
			copy(buf.b[33*k:], p[:])
		}
		if C.gv_keys_load(g.ctx, C.size_t(len(fresh)), (*C.uint8_t)(buf.p), (*C.uint32_t)(out.p)) == 0 {
			s := (*[maxBatchBytes / 4]uint32)(out.p)[:len(fresh):len(fresh)]
			for k, p := range fresh {
				g.slots[p] = s[k]
			}
		}
	}
	for i, p := range pubs {
		if s, ok := g.slots[p]; ok {
			slots[i], loaded[i] = s, true
		}
	}
	return slots, loaded
}

// ResetKeys empties the key arena and the slot map together (a slot number
// must never outlive the arena row it names).
func (g *GPU) ResetKeys() {
	g.mu.Lock()
	defer g.mu.Unlock()
	C.gv_keys_reset(g.ctx)
	g.slots = map[secp256k1.PubKeySecp256k1]uint32{}
	g.slotGen = uint64(C.gv_keys_generation(g.ctx))
}

// VerifyBatchKeyed is VerifyBatch with the keys kept parsed in HBM: every
// key is parsed (decompressed, tabulated) once and verified by slot.  Same
// verdicts; leaves whose key could not be cached go to the CPU.
func (g *GPU) VerifyBatchKeyed(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
	n := len(pubs)
	ok := make([]bool, n)
	slots, loaded := g.slotsFor(pubs)
	idx := make([]int, 0, n)
	total := 0
	for i := range pubs {
		if len(sigs[i]) != 64 {
			continue
		}
		if !loaded[i] {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i])
			continue
		}
		idx = append(idx, i)
		total += len(msgs[i])
	}
	if len(idx) == 0 {
		return ok
	}
	m := len(idx)
	sl, sig, blob, off, ln, out := newCBuf(4*m), newCBuf(64*m), newCBuf(total), newCBuf(8*m), newCBuf(4*m), newCBuf(m)
	defer func() { sl.free(); sig.free(); blob.free(); off.free(); ln.free(); out.free() }()
	s := (*[maxBatchBytes / 4]uint32)(sl.p)[:m:m]
	o := (*[maxBatchBytes / 8]uint64)(off.p)[:m:m]
	l := (*[maxBatchBytes / 4]uint32)(ln.p)[:m:m]
	pos := 0
	for k, i := range idx {
		s[k] = slots[i]
		copy(sig.b[64*k:], sigs[i])
		o[k], l[k] = uint64(pos), uint32(len(msgs[i]))
		pos += copy(blob.b[pos:], msgs[i])
	}
	// the arena may not be reset while a keyed verify runs (gpuverify.h)
	g.mu.Lock()
	rc := C.gv_verify_msgs_keyed(g.ctx, C.size_t(m), (*C.uint32_t)(sl.p), (*C.uint8_t)(sig.p), (*C.uint8_t)(blob.p),
		(*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
	g.mu.Unlock()
	for k, i := range idx {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i])
		}
	}
	return ok
}
