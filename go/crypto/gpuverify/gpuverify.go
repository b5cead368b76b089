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
	"math/bits"
	"os"
	"strconv"
	"sync"
	"sync/atomic"
	"time"
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

// AsyncVerifier queues a batch and returns at once: wait returns the
// verdicts (VerifyBatch's).  wait is idempotent -- later calls return the
// first call's verdicts -- so a caller can defer it as a guard: a batch that
// is never waited keeps its pinned buffers out of the pool (GPU.Close would
// block on them) and its ticket in the library.  The GPU implements it with
// gv_submit_msgs[_keyed] / gv_wait, so the batch runs while the caller does
// other work -- the same block's ed25519 leaves, the next block's state stage
// -- and consecutive batches run as one stream of chunks on the device.
type AsyncVerifier interface {
	SubmitBatch(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) (wait func() []bool)
}

// EdKeyCache is an EdVerifier that can keep a key set resident whatever the
// batch size: a light client's validator set signs block after block, so its
// keys are parsed and tabulated once (gv_ed_keys_load) and every later commit
// runs on the cached-key kernel (~0.08 ms for 64 signatures against ~1 ms).
// Same verdicts as VerifyBatchEd25519.
type EdKeyCache interface {
	EdVerifier
	VerifyBatchEd25519Cached(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool
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

// Routing defaults, shared with the C++ mirror through gpuverify.h so the
// two cannot drift apart (tests/test_go_policy.py checks both use them).
var (
	DefaultCPUBelow   = int(C.GV_CPU_CROSSOVER) // batches below: the reference VerifyBytes on the CPU
	DefaultKeyLoadMin = int(C.GV_KEY_LOAD_MIN)  // batches from: keys not yet resident are loaded
	DefaultKeyCap     = int(C.GV_KEY_CAP)       // key-arena size at which it is reset
	DefaultEdKeyCap   = int(C.GV_ED_KEY_CAP)    // ed25519 key-arena size at which it is reset
)

// envInt: a positive integer from the environment, else def.
func envInt(name string, def int) int {
	if v, err := strconv.Atoi(os.Getenv(name)); err == nil && v > 0 {
		return v
	}
	return def
}

// Logger is the subset of tendermint's libs/log.Logger the shim reports
// through (baseapp.go:44 keeps one per app): a device failure is logged once
// per fallback call, with the batch size and the library's error string.
type Logger interface {
	Error(msg string, keyvals ...interface{})
}

// Stats counts what the shim did since Open (SURVEY.md §5: GPU vs CPU
// fallback, batch sizes, latency).  Histograms are log2 buckets: bucket k
// holds values in [2^k, 2^(k+1)) (batch leaves; call latency in us).
type Stats struct {
	GPUCalls, GPULeaves             uint64 // library calls that answered, and their leaves
	CPURouted, CPURoutedLeaves      uint64 // batches below CPUBelow: the reference VerifyBytes by policy
	FallbackCalls, FallbackLeaves   uint64 // library errors: leaves re-verified on the CPU (fail closed)
	KeyedCalls, Pub33Calls, EdCalls uint64
	KeyLoads, KeyResets             uint64
	BatchLog2                       [24]uint64
	LatencyUsLog2                   [24]uint64
}

type counters struct {
	gpuCalls, gpuLeaves, cpuRouted, cpuRoutedLeaves, fbCalls, fbLeaves uint64
	keyed, pub33, ed, keyLoads, keyResets                             uint64
	batch, lat                                                        [24]uint64
}

func log2b(v uint64) int {
	if v == 0 {
		return 0
	}
	k := bits.Len64(v) - 1
	if k > 23 {
		k = 23
	}
	return k
}

// done records one library call of n leaves that took d; rc != 0 is a
// fallback (the leaves were re-verified on the CPU).
func (g *GPU) done(what string, n int, d time.Duration, rc C.int) {
	c := &g.cnt
	atomic.AddUint64(&c.batch[log2b(uint64(n))], 1)
	if rc == 0 {
		atomic.AddUint64(&c.gpuCalls, 1)
		atomic.AddUint64(&c.gpuLeaves, uint64(n))
		atomic.AddUint64(&c.lat[log2b(uint64(d.Microseconds()))], 1)
		return
	}
	atomic.AddUint64(&c.fbCalls, 1)
	atomic.AddUint64(&c.fbLeaves, uint64(n))
	if g.Logger != nil {
		g.Logger.Error("gpuverify: device call failed, leaves re-verified on the CPU", "call", what, "leaves", n,
			"err", C.GoString(C.gv_strerror(rc)))
	}
}

// Stats returns a snapshot of the counters.
func (g *GPU) Stats() Stats {
	c := &g.cnt
	s := Stats{
		GPUCalls: atomic.LoadUint64(&c.gpuCalls), GPULeaves: atomic.LoadUint64(&c.gpuLeaves),
		CPURouted: atomic.LoadUint64(&c.cpuRouted), CPURoutedLeaves: atomic.LoadUint64(&c.cpuRoutedLeaves),
		FallbackCalls: atomic.LoadUint64(&c.fbCalls), FallbackLeaves: atomic.LoadUint64(&c.fbLeaves),
		KeyedCalls: atomic.LoadUint64(&c.keyed), Pub33Calls: atomic.LoadUint64(&c.pub33),
		EdCalls: atomic.LoadUint64(&c.ed), KeyLoads: atomic.LoadUint64(&c.keyLoads),
		KeyResets: atomic.LoadUint64(&c.keyResets),
	}
	for k := range s.BatchLog2 {
		s.BatchLog2[k] = atomic.LoadUint64(&c.batch[k])
		s.LatencyUsLog2[k] = atomic.LoadUint64(&c.lat[k])
	}
	return s
}

// GPU is a libgpuverify context on one or more HIP devices.  Safe for
// concurrent use: the library serialises calls per device, and the key-cache
// maps below are guarded by mu.
//
// VerifyBatch (what BatchSigVerificationDecorator and NewPreVerifier call)
// routes every batch by the policy below, the policy of the tested C++ mirror
// (host/gvhost.cpp verify_secp): fewer than CPUBelow leaves -> the reference
// VerifyBytes on the CPU; Keyed and every key resident -> the key-arena path;
// Keyed and at least KeyLoadMin leaves -> the new keys are loaded once, then
// the key-arena path; otherwise the pub33 path.  Same verdicts on every route.
type GPU struct {
	ctx       *C.gv_ctx
	closeOnce sync.Once

	// CPUBelow: below the measured crossover a VerifyBytes loop answers first
	// (one core: ~0.20 ms per signature; the sliced small-batch kernels:
	// ~0.21 ms for up to 256 signatures, DESIGN.md §6.3).
	CPUBelow int
	// Keyed: verify through the context's key arena (the account pubkey cache,
	// SURVEY.md §8f-2: 197M/s vs 103M/s at 1M, 0.10 vs 0.21 ms at 64).
	Keyed bool
	// KeyLoadMin: the smallest batch that loads keys (k_keys_build costs about
	// a millisecond; a CheckTx batch never waits on it).
	KeyLoadMin int
	// KeyCap: the arena is reset when a load would take it past this many keys.
	KeyCap int
	// EdKeyCap: the same for the ed25519 key arena (72 KB of HBM per key;
	// default GV_ED_KEY_CAP, env GV_ED_KEY_CAP).
	EdKeyCap int
	// Logger, when set, reports every call that fell back to the CPU.
	Logger Logger

	cnt  counters
	pool pinnedPool

	mu      sync.Mutex                           // the slot maps AND every keyed call (no reset in between)
	slots   map[secp256k1.PubKeySecp256k1]uint32 // key -> key-arena slot (gv_keys_load)
	slotGen uint64                               // gv_keys_generation the slot map belongs to
	edSlots map[ed25519.PubKeyEd25519]uint32     // ed25519 key -> ed25519 key-arena slot (gv_ed_keys_load)
	edGen   uint64                               // gv_ed_keys_generation the ed25519 map belongs to
}

var (
	_ Verifier   = (*GPU)(nil)
	_ EdVerifier = (*GPU)(nil)
	_ EdKeyCache = (*GPU)(nil)
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
	g := &GPU{ctx: ctx, CPUBelow: DefaultCPUBelow, Keyed: true, KeyLoadMin: DefaultKeyLoadMin,
		KeyCap: envInt("GV_KEY_CAP", DefaultKeyCap), EdKeyCap: envInt("GV_ED_KEY_CAP", DefaultEdKeyCap),
		slots: map[secp256k1.PubKeySecp256k1]uint32{}, edSlots: map[ed25519.PubKeyEd25519]uint32{}}
	g.pool.ctx = ctx
	// the library's arena growth doubles up to the reset points the shim uses
	// (past them it grows to exactly what is needed, no quadratic copying)
	if err := g.SetOption("key_cap", int64(g.KeyCap)); err != nil {
		g.Close()
		return nil, err
	}
	if err := g.SetOption("ed_key_cap", int64(g.EdKeyCap)); err != nil {
		g.Close()
		return nil, err
	}
	return g, nil
}

// Close releases the pinned buffers and the context (idempotent).  It first
// waits for the pinned buffers that in-flight calls still hold: they go back
// to the pool while the context is valid (gv_host_free needs it), and no new
// pinned buffer is handed out once closing has begun.
func (g *GPU) Close() {
	g.closeOnce.Do(func() {
		g.pool.close()
		C.gv_close(g.ctx)
	})
}

// SetOption forwards to gv_set_option ("max_batch", "lat_max", "pipe_chunk", ...).
func (g *GPU) SetOption(key string, val int64) error {
	ck := C.CString(key)
	defer C.free(unsafe.Pointer(ck))
	if rc := C.gv_set_option(g.ctx, ck, C.longlong(val)); rc != 0 {
		return errors.New("gpuverify: gv_set_option(" + key + "): " + C.GoString(C.gv_strerror(rc)))
	}
	return nil
}

// cbuf is a C allocation viewed as a Go byte slice (returned by free()).
// Batch buffers come from the context's pinned host memory (gv_host_alloc):
// the library reads such inputs in place (DMA, or zero-copy for small
// batches) instead of staging pageable memory through its copy pool, which
// cost ~47 % of the device rate on one GPU (DESIGN.md §6.4).  They are
// recycled by power-of-two size class; a failed pinned allocation falls back
// to C.malloc (the library then stages it, same verdicts).
type cbuf struct {
	p     unsafe.Pointer
	b     []byte
	class int // size class (pinned), -1: C.malloc
	pool  *pinnedPool
}

// pinnedPool: free lists of gv_host_alloc buffers per size class 2^k bytes,
// at most pinnedKeep bytes parked in all.
type pinnedPool struct {
	ctx     *C.gv_ctx
	mu      sync.Mutex
	free    [32][]unsafe.Pointer
	parked  int
	out     int        // pinned buffers handed out and not yet returned
	closing bool       // Close has begun: get() hands out C.malloc buffers only
	idle    *sync.Cond // signalled when out drops to 0 while closing
}

const pinnedKeep = 1 << 30

func (p *pinnedPool) get(n int) cbuf {
	k := bits.Len(uint(n - 1))
	if k < 12 {
		k = 12 // 4 KiB minimum class
	}
	if k < 32 {
		p.mu.Lock()
		if p.closing {
			p.mu.Unlock()
		} else if l := len(p.free[k]); l > 0 {
			ptr := p.free[k][l-1]
			p.free[k] = p.free[k][:l-1]
			p.parked -= 1 << k
			p.out++
			p.mu.Unlock()
			return cbuf{ptr, (*[maxBatchBytes]byte)(ptr)[:n:n], k, p}
		} else {
			p.out++ // reserved before the allocation, so Close waits for it
			p.mu.Unlock()
			var ptr unsafe.Pointer
			if p.ctx != nil && C.gv_host_alloc(p.ctx, C.size_t(1)<<uint(k), &ptr) == 0 {
				return cbuf{ptr, (*[maxBatchBytes]byte)(ptr)[:n:n], k, p}
			}
			p.mu.Lock()
			p.release()
			p.mu.Unlock()
		}
	}
	ptr := C.malloc(C.size_t(n))
	return cbuf{ptr, (*[maxBatchBytes]byte)(ptr)[:n:n], -1, nil}
}

// release: one handed-out buffer is back (p.mu held).
func (p *pinnedPool) release() {
	p.out--
	if p.out == 0 && p.closing && p.idle != nil {
		p.idle.Broadcast()
	}
}

func (p *pinnedPool) put(c cbuf) {
	p.mu.Lock()
	defer p.mu.Unlock()
	if !p.closing && p.parked+(1<<c.class) <= pinnedKeep {
		p.free[c.class] = append(p.free[c.class], c.p)
		p.parked += 1 << c.class
	} else {
		C.gv_host_free(p.ctx, c.p) // Close is waiting for this buffer: the context is still open
	}
	p.release()
}

// close: no more pinned buffers out, wait for the outstanding ones, free
// every parked buffer.  The context stays open until it returns.
func (p *pinnedPool) close() {
	p.mu.Lock()
	defer p.mu.Unlock()
	p.closing = true
	if p.idle == nil {
		p.idle = sync.NewCond(&p.mu)
	}
	for p.out > 0 {
		p.idle.Wait()
	}
	for k := range p.free {
		for _, ptr := range p.free[k] {
			C.gv_host_free(p.ctx, ptr)
		}
		p.free[k] = nil
	}
	p.parked = 0
}

func (g *GPU) newCBuf(n int) cbuf {
	if n < 1 {
		n = 1
	}
	return g.pool.get(n)
}

func (c cbuf) free() {
	if c.class < 0 {
		C.free(c.p)
		return
	}
	c.pool.put(c)
}

// VerifyBatch implements Verifier with the routing policy of the GPU type.
func (g *GPU) VerifyBatch(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
	if len(pubs) < g.CPUBelow {
		atomic.AddUint64(&g.cnt.cpuRouted, 1)
		atomic.AddUint64(&g.cnt.cpuRoutedLeaves, uint64(len(pubs)))
		return CPU{}.VerifyBatch(pubs, msgs, sigs)
	}
	if g.Keyed {
		return g.VerifyBatchKeyed(pubs, msgs, sigs)
	}
	return g.VerifyBatchPub33(pubs, msgs, sigs)
}

// VerifyBatchPub33: every leaf with its compressed key (gv_verify_msgs).
// Leaves whose signature is not 64 bytes are false without reaching the GPU
// (VerifyBytes' first check).  On any nonzero return the whole call is
// re-verified on the CPU.
func (g *GPU) VerifyBatchPub33(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
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
		copy(ok, g.VerifyBatchPub33(pubs[:h], msgs[:h], sigs[:h]))
		copy(ok[h:], g.VerifyBatchPub33(pubs[h:], msgs[h:], sigs[h:]))
		return ok
	}
	m := len(idx)
	pub, sig, blob, off, ln, out := g.newCBuf(33*m), g.newCBuf(64*m), g.newCBuf(total), g.newCBuf(8*m), g.newCBuf(4*m), g.newCBuf(m)
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
	t0 := time.Now()
	rc := C.gv_verify_msgs(g.ctx, C.size_t(m), (*C.uint8_t)(pub.p), (*C.uint8_t)(sig.p), (*C.uint8_t)(blob.p),
		(*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
	atomic.AddUint64(&g.cnt.pub33, 1)
	g.done("gv_verify_msgs", m, time.Since(t0), rc)
	for k, i := range idx {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
		}
	}
	return ok
}

// VerifyBatchEd25519 implements EdVerifier (go1.14 crypto/ed25519 semantics
// on the GPU) with the secp256k1 routing rule: Keyed and every key resident,
// or at least KeyLoadMin leaves -> the ed25519 key arena (the host mirror's
// verify_ed); otherwise every leaf with its key.  Same verdicts either way.
func (g *GPU) VerifyBatchEd25519(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool {
	if g.Keyed {
		return g.verifyEdKeyed(pubs, msgs, sigs, len(pubs) >= g.KeyLoadMin)
	}
	return g.VerifyBatchEd25519Pub(pubs, msgs, sigs)
}

// VerifyBatchEd25519Cached implements EdKeyCache: the keys not resident are
// loaded whatever the batch size (a validator set).
func (g *GPU) VerifyBatchEd25519Cached(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool {
	return g.verifyEdKeyed(pubs, msgs, sigs, true)
}

// VerifyBatchEd25519Pub: every leaf with its 32-byte key
// (gv_verify_ed25519_msgs).  Same fail-closed rule as VerifyBatch.
func (g *GPU) VerifyBatchEd25519Pub(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte) []bool {
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
		copy(ok, g.VerifyBatchEd25519Pub(pubs[:h], msgs[:h], sigs[:h]))
		copy(ok[h:], g.VerifyBatchEd25519Pub(pubs[h:], msgs[h:], sigs[h:]))
		return ok
	}
	m := len(idx)
	pub, sig, blob, off, ln, out := g.newCBuf(32*m), g.newCBuf(64*m), g.newCBuf(total), g.newCBuf(8*m), g.newCBuf(4*m), g.newCBuf(m)
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
	t0 := time.Now()
	rc := C.gv_verify_ed25519_msgs(g.ctx, C.size_t(m), (*C.uint8_t)(pub.p), (*C.uint8_t)(sig.p), (*C.uint8_t)(blob.p),
		(*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
	atomic.AddUint64(&g.cnt.ed, 1)
	g.done("gv_verify_ed25519_msgs", m, time.Since(t0), rc)
	for k, i := range idx {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
		}
	}
	return ok
}


// SubmitBatch implements AsyncVerifier with VerifyBatch's routing (CPU below
// CPUBelow, keyed leaves by arena slot, the rest by pub33) and fail-closed
// rule.  g.mu is held from the slot lookup through the submission: once
// queued, a batch needs no lock -- the library runs every queued batch
// before a gv_keys_load / gv_keys_reset moves a slot.  The pinned buffers
// stay referenced until wait returns (the library reads them until gv_wait).
func (g *GPU) SubmitBatch(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) func() []bool {
	n := len(pubs)
	idx := make([]int, 0, n)
	total := 0
	for i := range pubs {
		if len(sigs[i]) == 64 { // VerifyBytes' first check
			idx = append(idx, i)
			total += len(msgs[i])
		}
	}
	if n < g.CPUBelow || len(idx) == 0 || total+97*len(idx) > maxBatchBytes {
		res := g.VerifyBatch(pubs, msgs, sigs) // nothing to overlap (CPU, empty) or split: synchronous
		return func() []bool { return res }
	}
	type queued struct {
		sel    []int
		ticket C.uint64_t
		rc     C.int
		out    cbuf
		bufs   []cbuf
		what   string
	}
	submit := func(sel []int, slots []uint32) *queued {
		m := len(sel)
		q := &queued{sel: sel}
		size := 0
		for _, i := range sel {
			size += len(msgs[i])
		}
		var key cbuf
		if slots != nil {
			key = g.newCBuf(4 * m)
		} else {
			key = g.newCBuf(33 * m)
		}
		sig, blob, off, ln := g.newCBuf(64*m), g.newCBuf(size), g.newCBuf(8*m), g.newCBuf(4*m)
		q.out = g.newCBuf(m)
		q.bufs = []cbuf{key, sig, blob, off, ln}
		o := (*[maxBatchBytes / 8]uint64)(off.p)[:m:m]
		l := (*[maxBatchBytes / 4]uint32)(ln.p)[:m:m]
		pos := 0
		for k, i := range sel {
			if slots != nil {
				(*[maxBatchBytes / 4]uint32)(key.p)[k] = slots[i]
			} else {
				copy(key.b[33*k:], pubs[i][:])
			}
			copy(sig.b[64*k:], sigs[i])
			o[k], l[k] = uint64(pos), uint32(len(msgs[i]))
			pos += copy(blob.b[pos:], msgs[i])
		}
		if slots != nil {
			q.what = "gv_submit_msgs_keyed"
			q.rc = C.gv_submit_msgs_keyed(g.ctx, C.size_t(m), (*C.uint32_t)(key.p), (*C.uint8_t)(sig.p),
				(*C.uint8_t)(blob.p), (*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(q.out.p), &q.ticket)
			atomic.AddUint64(&g.cnt.keyed, 1)
		} else {
			q.what = "gv_submit_msgs"
			q.rc = C.gv_submit_msgs(g.ctx, C.size_t(m), (*C.uint8_t)(key.p), (*C.uint8_t)(sig.p),
				(*C.uint8_t)(blob.p), (*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(q.out.p), &q.ticket)
			atomic.AddUint64(&g.cnt.pub33, 1)
		}
		return q
	}
	var qs []*queued
	if g.Keyed {
		g.mu.Lock()
		slots, loaded, _ := g.slotsLocked(pubs, n >= g.KeyLoadMin)
		var keyed, rest []int
		for _, i := range idx {
			if loaded[i] {
				keyed = append(keyed, i)
			} else {
				rest = append(rest, i)
			}
		}
		if len(keyed) > 0 {
			qs = append(qs, submit(keyed, slots))
		}
		g.mu.Unlock()
		if len(rest) > 0 {
			qs = append(qs, submit(rest, nil))
		}
	} else {
		qs = append(qs, submit(idx, nil))
	}
	t0 := time.Now()
	var once sync.Once
	var verdicts []bool
	waitAll := func() []bool {
		ok := make([]bool, n)
		for _, q := range qs {
			rc := q.rc
			if rc == 0 {
				rc = C.gv_wait(g.ctx, q.ticket)
			}
			g.done(q.what, len(q.sel), time.Since(t0), rc)
			for k, i := range q.sel {
				if rc == 0 {
					ok[i] = q.out.b[k] == 1
				} else {
					ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
				}
			}
			for _, b := range q.bufs {
				b.free()
			}
			q.out.free()
		}
		return ok
	}
	return func() []bool {
		once.Do(func() { verdicts = waitAll() })
		return verdicts
	}
}

// ---- account key cache (gv_keys_load, SURVEY.md §8f-2)

// slotsLocked returns each key's arena slot (g.mu held).  Keys not resident
// are loaded with ONE gv_keys_load when load is true; loaded[i] is false for
// a key that is not resident afterwards (not loaded, or the load failed):
// the caller verifies that leaf by pub33 -- never a sentinel slot, whose
// keyed verify would read as a rejection.
func (g *GPU) slotsLocked(pubs []secp256k1.PubKeySecp256k1, load bool) (slots []uint32, loaded []bool, all bool) {
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
	if len(fresh) == 0 {
		return slots, loaded, true
	}
	if !load {
		return slots, loaded, false
	}
	if int(C.gv_keys_count(g.ctx))+len(fresh) > g.KeyCap { // start the arena over (the C++ mirror's rule)
		atomic.AddUint64(&g.cnt.keyResets, 1)
		C.gv_keys_reset(g.ctx)
		g.slots = map[secp256k1.PubKeySecp256k1]uint32{}
		g.slotGen = uint64(C.gv_keys_generation(g.ctx))
		return g.slotsLocked(pubs, len(pubs) <= g.KeyCap)
	}
	buf := g.newCBuf(33 * len(fresh))
	out := g.newCBuf(4 * len(fresh))
	defer func() { buf.free(); out.free() }()
	for k, p := range fresh {
		copy(buf.b[33*k:], p[:])
	}
	atomic.AddUint64(&g.cnt.keyLoads, 1)
	if C.gv_keys_load(g.ctx, C.size_t(len(fresh)), (*C.uint8_t)(buf.p), (*C.uint32_t)(out.p)) == 0 {
		s := (*[maxBatchBytes / 4]uint32)(out.p)[:len(fresh):len(fresh)]
		for k, p := range fresh {
			g.slots[p] = s[k]
		}
	}
	all = true
	for i, p := range pubs {
		if s, ok := g.slots[p]; ok {
			slots[i], loaded[i] = s, true
		} else {
			all = false
		}
	}
	return slots, loaded, all
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

// VerifyBatchKeyed is VerifyBatchPub33 with the keys kept parsed in HBM:
// every key is parsed (decompressed, tabulated) once and verified by slot.
// Same verdicts.  Keys not resident are loaded only by batches of at least
// KeyLoadMin leaves; the leaves of keys that are not resident go by pub33.
// g.mu is held from the slot lookup through the keyed verify, so no
// ResetKeys or reload can move a slot in between.
func (g *GPU) VerifyBatchKeyed(pubs []secp256k1.PubKeySecp256k1, msgs, sigs [][]byte) []bool {
	n := len(pubs)
	ok := make([]bool, n)
	idx := make([]int, 0, n)
	total := 0
	for i := range pubs {
		if len(sigs[i]) == 64 { // VerifyBytes' first check
			idx = append(idx, i)
			total += len(msgs[i])
		}
	}
	if len(idx) == 0 {
		return ok
	}
	if total+76*len(idx) > maxBatchBytes { // split oversize batches
		h := n / 2
		copy(ok, g.VerifyBatchKeyed(pubs[:h], msgs[:h], sigs[:h]))
		copy(ok[h:], g.VerifyBatchKeyed(pubs[h:], msgs[h:], sigs[h:]))
		return ok
	}
	g.mu.Lock()
	slots, loaded, _ := g.slotsLocked(pubs, n >= g.KeyLoadMin)
	var rest []int // leaves whose key is not resident: pub33
	keyed := idx[:0:0]
	for _, i := range idx {
		if loaded[i] {
			keyed = append(keyed, i)
		} else {
			rest = append(rest, i)
		}
	}
	rc := C.int(0)
	var out cbuf
	if len(keyed) > 0 {
		m := len(keyed)
		sl, sig, blob, off, ln := g.newCBuf(4*m), g.newCBuf(64*m), g.newCBuf(total), g.newCBuf(8*m), g.newCBuf(4*m)
		out = g.newCBuf(m)
		s := (*[maxBatchBytes / 4]uint32)(sl.p)[:m:m]
		o := (*[maxBatchBytes / 8]uint64)(off.p)[:m:m]
		l := (*[maxBatchBytes / 4]uint32)(ln.p)[:m:m]
		pos := 0
		for k, i := range keyed {
			s[k] = slots[i]
			copy(sig.b[64*k:], sigs[i])
			o[k], l[k] = uint64(pos), uint32(len(msgs[i]))
			pos += copy(blob.b[pos:], msgs[i])
		}
		t0 := time.Now()
		rc = C.gv_verify_msgs_keyed(g.ctx, C.size_t(m), (*C.uint32_t)(sl.p), (*C.uint8_t)(sig.p), (*C.uint8_t)(blob.p),
			(*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
		atomic.AddUint64(&g.cnt.keyed, 1)
		g.done("gv_verify_msgs_keyed", m, time.Since(t0), rc)
		sl.free()
		sig.free()
		blob.free()
		off.free()
		ln.free()
	}
	g.mu.Unlock()
	for k, i := range keyed {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
		}
	}
	if len(keyed) > 0 {
		out.free()
	}
	if len(rest) > 0 {
		p := make([]secp256k1.PubKeySecp256k1, len(rest))
		ms := make([][]byte, len(rest))
		ss := make([][]byte, len(rest))
		for k, i := range rest {
			p[k], ms[k], ss[k] = pubs[i], msgs[i], sigs[i]
		}
		for k, v := range g.VerifyBatchPub33(p, ms, ss) {
			ok[rest[k]] = v
		}
	}
	return ok
}

// ---- ed25519 key cache (gv_ed_keys_load)

// edSlotsLocked returns each key's ed25519 arena slot (g.mu held), loading
// the keys not resident with ONE gv_ed_keys_load when load is true; all is
// false when some key is not resident afterwards.
func (g *GPU) edSlotsLocked(pubs []ed25519.PubKeyEd25519, load bool) (slots []uint32, all bool) {
	if gen := uint64(C.gv_ed_keys_generation(g.ctx)); gen != g.edGen {
		g.edSlots = map[ed25519.PubKeyEd25519]uint32{}
		g.edGen = gen
	}
	slots = make([]uint32, len(pubs))
	var fresh []ed25519.PubKeyEd25519
	seen := map[ed25519.PubKeyEd25519]bool{}
	for i, p := range pubs {
		if s, ok := g.edSlots[p]; ok {
			slots[i] = s
		} else if !seen[p] {
			seen[p] = true
			fresh = append(fresh, p)
		}
	}
	if len(fresh) == 0 {
		return slots, true
	}
	if !load || len(fresh) > g.EdKeyCap {
		return slots, false
	}
	if int(C.gv_ed_keys_count(g.ctx))+len(fresh) > g.EdKeyCap { // start the arena over (the C++ mirror's rule)
		atomic.AddUint64(&g.cnt.keyResets, 1)
		C.gv_ed_keys_reset(g.ctx)
		g.edSlots = map[ed25519.PubKeyEd25519]uint32{}
		g.edGen = uint64(C.gv_ed_keys_generation(g.ctx))
		return g.edSlotsLocked(pubs, true)
	}
	buf := g.newCBuf(32 * len(fresh))
	out := g.newCBuf(4 * len(fresh))
	defer func() { buf.free(); out.free() }()
	for k, p := range fresh {
		copy(buf.b[32*k:], p[:])
	}
	atomic.AddUint64(&g.cnt.keyLoads, 1)
	if C.gv_ed_keys_load(g.ctx, C.size_t(len(fresh)), (*C.uint8_t)(buf.p), (*C.uint32_t)(out.p)) != 0 {
		return slots, false
	}
	s := (*[maxBatchBytes / 4]uint32)(out.p)[:len(fresh):len(fresh)]
	for k, p := range fresh {
		g.edSlots[p] = s[k]
	}
	for i, p := range pubs {
		slots[i] = g.edSlots[p]
	}
	return slots, true
}

// verifyEdKeyed: the leaves by ed25519 arena slot (gv_verify_ed25519_msgs_keyed)
// when every key is (or, with load, becomes) resident, else the unkeyed batch.
// g.mu is held from the slot lookup through the verify.
func (g *GPU) verifyEdKeyed(pubs []ed25519.PubKeyEd25519, msgs, sigs [][]byte, load bool) []bool {
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
	if total+76*len(idx) > maxBatchBytes { // split oversize batches
		h := n / 2
		copy(ok, g.verifyEdKeyed(pubs[:h], msgs[:h], sigs[:h], load))
		copy(ok[h:], g.verifyEdKeyed(pubs[h:], msgs[h:], sigs[h:], load))
		return ok
	}
	sub := make([]ed25519.PubKeyEd25519, len(idx))
	for k, i := range idx {
		sub[k] = pubs[i]
	}
	g.mu.Lock()
	slots, all := g.edSlotsLocked(sub, load)
	if !all {
		g.mu.Unlock()
		return g.VerifyBatchEd25519Pub(pubs, msgs, sigs)
	}
	m := len(idx)
	sl, sig, blob, off, ln, out := g.newCBuf(4*m), g.newCBuf(64*m), g.newCBuf(total), g.newCBuf(8*m), g.newCBuf(4*m), g.newCBuf(m)
	defer func() { sl.free(); sig.free(); blob.free(); off.free(); ln.free(); out.free() }()
	sv := (*[maxBatchBytes / 4]uint32)(sl.p)[:m:m]
	o := (*[maxBatchBytes / 8]uint64)(off.p)[:m:m]
	l := (*[maxBatchBytes / 4]uint32)(ln.p)[:m:m]
	pos := 0
	for k, i := range idx {
		sv[k] = slots[k]
		copy(sig.b[64*k:], sigs[i])
		o[k], l[k] = uint64(pos), uint32(len(msgs[i]))
		pos += copy(blob.b[pos:], msgs[i])
	}
	t0 := time.Now()
	rc := C.gv_verify_ed25519_msgs_keyed(g.ctx, C.size_t(m), (*C.uint32_t)(sl.p), (*C.uint8_t)(sig.p),
		(*C.uint8_t)(blob.p), (*C.uint64_t)(off.p), (*C.uint32_t)(ln.p), (*C.uint8_t)(out.p))
	g.mu.Unlock()
	atomic.AddUint64(&g.cnt.ed, 1)
	g.done("gv_verify_ed25519_msgs_keyed", m, time.Since(t0), rc)
	for k, i := range idx {
		if rc == 0 {
			ok[i] = out.b[k] == 1
		} else {
			ok[i] = pubs[i].VerifyBytes(msgs[i], sigs[i]) // fail closed to the reference path
		}
	}
	return ok
}
