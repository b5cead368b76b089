package ante

// BatchSigVerificationDecorator: the drop-in for SigVerificationDecorator
// (x/auth/ante/sigverify.go:160-216) that verifies all of a transaction's
// signature leaves in one batch (verdict cache first, then the GPU through
// crypto/gpuverify), and NewPreVerifier, the block / mempool hook that fills
// the verdict cache ahead of the ante handler (SURVEY.md §8b, §8f-1).
//
// Same API, same error types and strings, same ReCheck / simulate bypass,
// same first-failure reporting order, and the same gas: the reference loop
// reads signer i's account through the gas-metered store only after signers
// 0..i-1 verified (sigverify.go:194-213; gaskv types/context.go:211-212,
// store/gaskv/store.go:36-43).  This decorator gathers the leaves through a
// look-ahead context whose gas meter is a fresh infinite one (nothing is
// charged to the tx), verifies them in one batch, and then walks the signers
// exactly as the reference loop does -- GetSignerAcc on the real context,
// verdict, return at the first failure -- so every read the tx is charged
// for is a read the reference makes, in the same order.  Wiring: replace
// NewSigVerificationDecorator(ak) at x/auth/ante/ante.go:27 with
// NewBatchSigVerificationDecorator(ak, verifier, cache).
//
// Source-level only in this repository (no Go toolchain in the build image);
// the C++ mirror host/gvhost.cpp implements the same logic and its gas is
// tested against a reference-order restatement (tests/test_gas_order.py).

import (
	"runtime"
	"sync"

	"github.com/tendermint/tendermint/crypto"
	"github.com/tendermint/tendermint/crypto/ed25519"
	"github.com/tendermint/tendermint/crypto/multisig"
	"github.com/tendermint/tendermint/crypto/secp256k1"

	"github.com/cosmos/cosmos-sdk/codec"
	gv "github.com/cosmos/cosmos-sdk/crypto/gpuverify"
	sdk "github.com/cosmos/cosmos-sdk/types"
	sdkerrors "github.com/cosmos/cosmos-sdk/types/errors"
	"github.com/cosmos/cosmos-sdk/x/auth/exported"
)

// BatchSigVerificationDecorator verifies every signer's signature of a tx
// with one batched call.
type BatchSigVerificationDecorator struct {
	ak    AccountKeeper
	v     gv.Verifier
	cache *gv.VerdictCache
}

// NewBatchSigVerificationDecorator: v verifies the cache misses (a *gv.GPU,
// or gv.CPU{}); cache may be nil (no cache).
func NewBatchSigVerificationDecorator(ak AccountKeeper, v gv.Verifier, cache *gv.VerdictCache) BatchSigVerificationDecorator {
	return BatchSigVerificationDecorator{ak: ak, v: v, cache: cache}
}

// AnteHandle implements sdk.AnteDecorator.
func (d BatchSigVerificationDecorator) AnteHandle(ctx sdk.Context, tx sdk.Tx, simulate bool, next sdk.AnteHandler) (sdk.Context, error) {
	// no need to verify signatures on recheck tx (sigverify.go:172)
	if ctx.IsReCheckTx() {
		return next(ctx, tx, simulate)
	}
	sigTx, ok := tx.(SigVerifiableTx)
	if !ok {
		return ctx, sdkerrors.Wrap(sdkerrors.ErrTxDecode, "invalid transaction type")
	}
	sigs := sigTx.GetSignatures()
	signerAddrs := sigTx.GetSigners()
	if len(sigs) != len(signerAddrs) { // sigverify.go:190-192
		return ctx, sdkerrors.Wrapf(sdkerrors.ErrUnauthorized, "invalid number of signer;  expected: %d, got %d", len(signerAddrs), len(sigs))
	}
	// Look-ahead: every signer's leaves up to the first signer the reference
	// loop would stop at, read through a context whose gas meter is not the
	// tx's, and all leaves answered at once.
	var b batch
	var exprs []*expr
	if !simulate { // sigverify.go:210: no verification when simulating
		exprs = d.gather(ctx.WithGasMeter(sdk.NewInfiniteGasMeter()), sigTx, sigs, signerAddrs, &b)
		b.resolve(d.v, d.cache)
	}
	// The reference loop (sigverify.go:194-213) on the real context.
	for i, sig := range sigs {
		acc, err := GetSignerAcc(ctx, d.ak, signerAddrs[i]) // gas-metered, as :195
		if err != nil {
			return ctx, err
		}
		// Sign bytes where the reference computes them (:201): after the
		// account read, before the nil-key check, and when simulating too.  A
		// gathered signer's bytes were computed by the look-ahead from the same
		// account and chain id (GetSignBytes reads nothing else), so only a
		// signer the look-ahead did not reach -- a nil key, a missing account
		// before it, or sign bytes that panicked -- recomputes them here, and
		// a Msg whose GetSignBytes panics panics at this point, as in the
		// reference (runTx turns it into ErrPanic).
		gathered := i < len(exprs) && exprs[i] != nil
		var signBytes []byte
		if !gathered {
			signBytes = sigTx.GetSignBytes(ctx, acc)
		}
		pubKey := acc.GetPubKey()
		if !simulate && pubKey == nil {
			return ctx, sdkerrors.Wrap(sdkerrors.ErrInvalidPubKey, "pubkey on account is not set")
		}
		if simulate {
			continue
		}
		var verified bool
		if gathered {
			verified = exprs[i].eval(&b)
		} else {
			verified = pubKey.VerifyBytes(signBytes, sig)
		}
		if !verified {
			return ctx, sdkerrors.Wrap(sdkerrors.ErrUnauthorized, "signature verification failed; verify correct account sequence and chain-id")
		}
	}
	return next(ctx, tx, simulate)
}

// gather builds signer i's verification expression for i = 0.. until the
// first signer whose account is missing or has no key (the loop reports it
// when it gets there) or whose sign bytes panic (the loop recomputes them on
// the real context and panics at the same point the reference does: before
// the nil-key check, sigverify.go:201-207).
func (d BatchSigVerificationDecorator) gather(look sdk.Context, sigTx SigVerifiableTx, sigs [][]byte,
	signerAddrs []sdk.AccAddress, b *batch) []*expr {
	exprs := make([]*expr, 0, len(sigs))
	for i, sig := range sigs {
		acc := d.ak.GetAccount(look, signerAddrs[i])
		if acc == nil {
			break
		}
		pubKey := acc.GetPubKey()
		if pubKey == nil {
			break
		}
		signBytes, ok := signBytesNoPanic(look, sigTx, acc)
		if !ok {
			break
		}
		exprs = append(exprs, b.build(pubKey, signBytes, sig))
	}
	return exprs
}

func signBytesNoPanic(ctx sdk.Context, sigTx SigVerifiableTx, acc exported.Account) (sb []byte, ok bool) {
	defer func() {
		if recover() != nil {
			sb, ok = nil, false
		}
	}()
	return sigTx.GetSignBytes(ctx, acc), true
}

// ---------------------------------------------------------------- leaves

// expr is pk.VerifyBytes(msg, sig) as an expression over leaves: a
// constant, one secp256k1 or ed25519 leaf, the AND of a multisig's set bits,
// or a deferred call for any other key (evaluated, on the CPU, only when the
// evaluation reaches it -- a nil multisig sub-key panics there and only
// there, after the sub-signatures before it passed, as in the reference).
type expr struct {
	konst  bool
	leaf   int // >= 0: index into batch.pubs (secp256k1)
	edLeaf int // >= 0: index into batch.ed (ed25519)
	and    []*expr
	isAnd  bool
	cpu    bool // deferred pk.VerifyBytes(msg, sig)
	pk     crypto.PubKey
	msg    []byte
	sig    []byte
}

func (e *expr) eval(b *batch) bool {
	switch {
	case e.cpu:
		return e.pk.VerifyBytes(e.msg, e.sig)
	case e.isAnd:
		for _, k := range e.and { // every leaf is a pure function: the AND equals the short-circuit
			if !k.eval(b) {
				return false
			}
		}
		return true
	case e.leaf >= 0:
		return b.ok[e.leaf]
	case e.edLeaf >= 0:
		return b.ed.ok[e.edLeaf]
	default:
		return e.konst
	}
}

type batch struct {
	pubs []secp256k1.PubKeySecp256k1
	msgs [][]byte
	sigs [][]byte
	keys [][32]byte
	ok   []bool
	ed   edBatch
}

type edBatch struct {
	pubs []ed25519.PubKeyEd25519
	msgs [][]byte
	sigs [][]byte
	ok   []bool
}

// build mirrors the key types the reference verifies (sigverify.go:303-321):
// secp256k1 and ed25519 leaves are batched; multisig (tendermint
// multisig.PubKeyMultisigThreshold.VerifyBytes) fans out in bit order with
// the same structural checks; any other key type verifies on the CPU.
func (b *batch) build(pk crypto.PubKey, msg, sig []byte) *expr {
	switch p := pk.(type) {
	case secp256k1.PubKeySecp256k1:
		if len(sig) != 64 { // VerifyBytes' first check
			return &expr{leaf: -1, edLeaf: -1}
		}
		b.pubs = append(b.pubs, p)
		b.msgs = append(b.msgs, msg)
		b.sigs = append(b.sigs, sig)
		return &expr{leaf: len(b.pubs) - 1, edLeaf: -1}
	case multisig.PubKeyMultisigThreshold:
		var ms multisig.Multisignature
		if err := codec.Cdc.UnmarshalBinaryBare(sig, &ms); err != nil {
			return &expr{leaf: -1, edLeaf: -1}
		}
		size := ms.BitArray.Size()
		if len(p.PubKeys) != size || len(ms.Sigs) < int(p.K) || len(ms.Sigs) > size ||
			ms.BitArray.NumTrueBitsBefore(size) < int(p.K) {
			return &expr{leaf: -1, edLeaf: -1}
		}
		e := &expr{leaf: -1, edLeaf: -1, isAnd: true}
		j := 0
		for i := 0; i < size; i++ {
			if ms.BitArray.GetIndex(i) {
				e.and = append(e.and, b.build(p.PubKeys[i], msg, ms.Sigs[j]))
				j++
			}
		}
		return e
	case ed25519.PubKeyEd25519:
		if len(sig) != 64 { // VerifyBytes' first check
			return &expr{leaf: -1, edLeaf: -1}
		}
		b.ed.pubs = append(b.ed.pubs, p)
		b.ed.msgs = append(b.ed.msgs, msg)
		b.ed.sigs = append(b.ed.sigs, sig)
		return &expr{leaf: -1, edLeaf: len(b.ed.pubs) - 1}
	default: // includes a nil sub-key: deferred to eval, which panics exactly where the reference does
		return &expr{leaf: -1, edLeaf: -1, cpu: true, pk: pk, msg: msg, sig: sig}
	}
}

// resolve answers every leaf: cache hits first, the misses in one Verifier
// call per key type (ed25519 through v's EdVerifier side when it has one),
// then the cache is filled.
//
// With an AsyncVerifier the secp256k1 misses are queued first and the ed25519
// leaves resolved while the GPU runs them.
func (b *batch) resolve(v gv.Verifier, cache *gv.VerdictCache) {
	av, async := v.(gv.AsyncVerifier)
	if !async {
		b.resolveEd(v, cache)
	}
	n := len(b.pubs)
	b.ok = make([]bool, n)
	b.keys = make([][32]byte, n)
	var miss []int
	for i := 0; i < n; i++ {
		b.keys[i] = gv.LeafKey(gv.KindSecp256k1, b.pubs[i][:], b.sigs[i], b.msgs[i])
		if cache != nil {
			if ok, hit := cache.Get(b.keys[i]); hit {
				b.ok[i] = ok
				continue
			}
		}
		miss = append(miss, i)
	}
	if len(miss) == 0 {
		if async {
			b.resolveEd(v, cache)
		}
		return
	}
	pubs := make([]secp256k1.PubKeySecp256k1, len(miss))
	msgs := make([][]byte, len(miss))
	sigs := make([][]byte, len(miss))
	for k, i := range miss {
		pubs[k], msgs[k], sigs[k] = b.pubs[i], b.msgs[i], b.sigs[i]
	}
	var res []bool
	if async {
		wait := av.SubmitBatch(pubs, msgs, sigs)
		// wait is idempotent: if resolveEd panics (the ante chain runs under
		// baseapp's recover) the queued batch is still waited for, so its
		// pinned buffers go back to the pool and GPU.Close does not block
		defer wait()
		b.resolveEd(v, cache) // beside the queued secp256k1 batch
		res = wait()
	} else {
		res = v.VerifyBatch(pubs, msgs, sigs)
	}
	for k, i := range miss {
		b.ok[i] = res[k]
		if cache != nil {
			cache.Put(b.keys[i], res[k])
		}
	}
}

func (b *batch) resolveEd(v gv.Verifier, cache *gv.VerdictCache) {
	e := &b.ed
	n := len(e.pubs)
	e.ok = make([]bool, n)
	keys := make([][32]byte, n)
	var miss []int
	for i := 0; i < n; i++ {
		keys[i] = gv.LeafKey(gv.KindEd25519, e.pubs[i][:], e.sigs[i], e.msgs[i])
		if cache != nil {
			if ok, hit := cache.Get(keys[i]); hit {
				e.ok[i] = ok
				continue
			}
		}
		miss = append(miss, i)
	}
	if len(miss) == 0 {
		return
	}
	ev, isEd := v.(gv.EdVerifier)
	if !isEd {
		ev = gv.CPU{}
	}
	pubs := make([]ed25519.PubKeyEd25519, len(miss))
	msgs := make([][]byte, len(miss))
	sigs := make([][]byte, len(miss))
	for k, i := range miss {
		pubs[k], msgs[k], sigs[k] = e.pubs[i], e.msgs[i], e.sigs[i]
	}
	res := ev.VerifyBatchEd25519(pubs, msgs, sigs)
	for k, i := range miss {
		e.ok[i] = res[k]
		if cache != nil {
			cache.Put(keys[i], res[k])
		}
	}
}

// ---------------------------------------------------------- PreVerifyTxs

// NewPreVerifier returns the function baseapp.PreVerifyTxs calls on a batch
// of decoded txs (a block before its DeliverTx loop, a mempool ingress batch,
// the genesis gentxs): every signer's sign bytes are predicted -- account
// number from state (0 at height 0, stdtx.go:249-253), sequence = state
// sequence + earlier txs of the same signer in the batch -- and all leaves
// are verified in one batch into the cache.  A wrong prediction is only a
// cache miss: the decorator rebuilds the sign bytes from the state it runs on.
//
// Two stages: the returned function reads the state (accounts, through a
// context with its own infinite gas meter) and returns the second stage,
// which touches no state -- sign bytes on every core, then the batch -- so a
// caller can release its state lock before the GPU call (baseapp Ingress).
func NewPreVerifier(ak AccountKeeper, v gv.Verifier, cache *gv.VerdictCache) func(ctx sdk.Context, txs []sdk.Tx) func() {
	ahead := NewPreVerifierAhead(ak, v, cache)
	return func(ctx sdk.Context, txs []sdk.Tx) func() { return ahead(ctx, nil, txs) }
}

// NewPreVerifierAhead is NewPreVerifier with a carry: txs that run before the
// batch but whose effects are not in ctx's state yet (block h while block h+1
// is pre-verified, baseapp.PreVerifyAhead).  Each carry tx advances every
// signer's predicted sequence by one (IncrementSequenceDecorator), and a key
// it supplies for an account without one is the key SetPubKeyDecorator will
// have stored -- the C++ mirror's carry (gvhost.cpp gvh_deliver_blocks: own,
// own_info).  The carry's leaves are not verified.
func NewPreVerifierAhead(ak AccountKeeper, v gv.Verifier, cache *gv.VerdictCache) func(ctx sdk.Context, carry, txs []sdk.Tx) func() {
	return func(ctx sdk.Context, carry, txs []sdk.Tx) func() {
		// Reads go through a context with its own infinite gas meter: the
		// hook runs outside any tx and must not charge a block or tx meter.
		look := ctx.WithGasMeter(sdk.NewInfiniteGasMeter())
		type job struct {
			sigTx SigVerifiableTx
			acc   exported.Account // this job's own decode, sequence set to the prediction
			pk    crypto.PubKey
			sig   []byte
		}
		var jobs []job
		bump := map[string]uint64{}
		stored := map[string]crypto.PubKey{} // keys the carry's SetPubKey stores
		for _, tx := range carry {
			sigTx, ok := tx.(SigVerifiableTx)
			if !ok {
				continue
			}
			signers, txPks := sigTx.GetSigners(), sigTx.GetPubKeys()
			for i, a := range signers {
				if i >= len(txPks) || txPks[i] == nil {
					continue
				}
				if _, have := stored[a.String()]; have {
					continue
				}
				if acc := ak.GetAccount(look, a); acc != nil && acc.GetPubKey() == nil {
					stored[a.String()] = txPks[i]
				}
			}
			for _, a := range signers {
				bump[a.String()]++
			}
		}
		for _, tx := range txs {
			sigTx, ok := tx.(SigVerifiableTx)
			if !ok {
				continue
			}
			sigs, signers, txPks := sigTx.GetSignatures(), sigTx.GetSigners(), sigTx.GetPubKeys()
			for i := 0; i < len(sigs) && i < len(signers); i++ {
				acc := ak.GetAccount(look, signers[i]) // a fresh decode: mutating it is local
				if acc == nil {
					continue
				}
				pk := acc.GetPubKey()
				if pk == nil {
					pk = stored[signers[i].String()] // stored by a carry tx's SetPubKey
				}
				if pk == nil && i < len(txPks) {
					pk = txPks[i] // SetPubKeyDecorator will store the tx-supplied key
				}
				if pk == nil {
					continue
				}
				_ = acc.SetSequence(acc.GetSequence() + bump[signers[i].String()])
				jobs = append(jobs, job{sigTx, acc, pk, sigs[i]})
			}
			for _, a := range signers {
				bump[a.String()]++
			}
		}
		// Sign bytes (JSON) on every core, then one batch.  The workers touch
		// no store and no gas meter: GetSignBytes reads only the chain id and
		// height of the context and the job's own account copy.
		if len(jobs) == 0 {
			return nil
		}
		return func() {
			parts := make([]batch, runtime.NumCPU())
			var wg sync.WaitGroup
			for w := range parts {
				wg.Add(1)
				go func(w int) {
					defer wg.Done()
					for k := w; k < len(jobs); k += len(parts) {
						j := jobs[k]
						func() {
							defer func() { _ = recover() }() // malformed tx: the ante chain reports it
							parts[w].build(j.pk, j.sigTx.GetSignBytes(look, j.acc), j.sig)
						}()
					}
				}(w)
			}
			wg.Wait()
			var all batch
			for _, p := range parts {
				all.pubs = append(all.pubs, p.pubs...)
				all.msgs = append(all.msgs, p.msgs...)
				all.sigs = append(all.sigs, p.sigs...)
				all.ed.pubs = append(all.ed.pubs, p.ed.pubs...)
				all.ed.msgs = append(all.ed.msgs, p.ed.msgs...)
				all.ed.sigs = append(all.ed.sigs, p.ed.sigs...)
			}
			all.resolve(v, cache)
		}
	}
}
