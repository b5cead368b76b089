package baseapp

// PreVerifyTxs and the mempool-side batching (SURVEY.md §8f-1): the hooks that
// fill the signature verdict cache the BatchSigVerificationDecorator reads
// (go/x/auth/ante/batch_sigverify.go).
//
// ABCI v0.33 hands the app one tx per DeliverTx / CheckTx
// (baseapp/abci.go:165-221), and the in-process node (server/start.go:173,
// proxy.NewLocalClientCreator) delivers them ONE AT A TIME under the local
// client's mutex -- the socket server serialises them too.  So a batch must be
// formed where txs actually queue up:
//   - a block: the executor calls PreVerifyTxs(block.Txs) after BeginBlock,
//     before its DeliverTx loop (the main batching path of a node);
//   - genesis: genutil.DeliverGenTxs (x/genutil/gentx.go:96-114) calls it on
//     the marshalled gentxs before delivering them;
//   - the mempool: Ingress takes txs where they arrive concurrently (RPC
//     broadcast handlers, the mempool reactor's Receive), before ABCI, and
//     pre-verifies them in batches without holding up CheckTx;
//   - CheckTxWindow batches CheckTx calls only when they DO arrive
//     concurrently (an application server that does not serialise them); a
//     lone call -- every call under the local client -- flushes at once and
//     waits for nothing.
// Nothing here changes a verdict: a missing or mispredicted cache entry is a
// miss and the decorator verifies it itself.
//
// One field is added to the BaseApp struct (baseapp/baseapp.go:45-92):
//
//	preVerifier PreVerifier // fills the signature verdict cache (SetPreVerifier)
//
// Source-level only in this repository (no Go toolchain in the build image);
// the C++ mirror (host/gvhost.cpp gvh_checktx) implements the same adaptive
// window and is measured (bench.py extras: checktx_serial).

import (
	"sync"
	"time"

	abci "github.com/tendermint/tendermint/abci/types"

	sdk "github.com/cosmos/cosmos-sdk/types"
)

// PreVerifier pre-verifies a batch of decoded txs against the state of ctx
// (x/auth/ante.NewPreVerifier).  It reads the state and returns the second,
// state-free stage (sign bytes + the verification batch + cache fill), so a
// caller may release its state lock before running it.  A nil second stage
// means nothing to do.
type PreVerifier func(ctx sdk.Context, txs []sdk.Tx) func()

// PreVerifierAhead is a PreVerifier whose sequence / key prediction also
// carries the effects of txs that precede the batch but are not in the state
// yet (x/auth/ante.NewPreVerifierAhead): every signer of a carry tx advances
// its sequence by one, and a key a carry tx supplies for an account that has
// none is the key its SetPubKeyDecorator stores.  The carry's own leaves are
// not verified.
type PreVerifierAhead func(ctx sdk.Context, carry, txs []sdk.Tx) func()

// SetPreVerifier registers the pre-verification hook (app construction,
// simapp/app.go:335-339, next to SetAnteHandler).
func (app *BaseApp) SetPreVerifier(pv PreVerifier) {
	if app.sealed {
		panic("SetPreVerifier() on sealed BaseApp")
	}
	app.preVerifier = pv
}

// SetPreVerifierAhead registers the block-replay hook (PreVerifyAhead).  One
// more BaseApp field: preVerifierAhead PreVerifierAhead.
func (app *BaseApp) SetPreVerifierAhead(pa PreVerifierAhead) {
	if app.sealed {
		panic("SetPreVerifierAhead() on sealed BaseApp")
	}
	app.preVerifierAhead = pa
}

func (app *BaseApp) decodeAll(txs [][]byte) []sdk.Tx {
	out := make([]sdk.Tx, 0, len(txs))
	for _, bz := range txs {
		if tx, err := app.txDecoder(bz); err == nil { // undecodable txs fail in DeliverTx as before
			out = append(out, tx)
		}
	}
	return out
}

// PreVerifyTxs pre-verifies a block's txs against the deliver state (call
// after BeginBlock, before the DeliverTx loop) or, before InitChain's
// deliver state exists, against the check state.
func (app *BaseApp) PreVerifyTxs(txs [][]byte) {
	if app.preVerifier == nil || len(txs) == 0 {
		return
	}
	st := app.deliverState
	if st == nil {
		st = app.checkState
	}
	if st == nil {
		return
	}
	if verify := app.preVerifier(st.ctx, app.decodeAll(txs)); verify != nil {
		verify()
	}
}

// PreVerifyAhead pipelines block replay (fast sync, catching up, the replay
// command -- wherever block h+1 is known while block h is delivered).  Call it
// after BeginBlock of block h and before h's first DeliverTx, with h's txs
// (cur) and h+1's (next): the state stage runs now, against the deliver state
// with cur's effects carried (they are not written yet), and the state-free
// stage -- sign bytes, the GPU batch, the cache fill -- runs on a goroutine
// beside h's DeliverTx loop.  Call the returned wait before BeginBlock of
// h+1.  A misprediction (a tx of block h that fails, so its signers'
// sequences do not advance) is only a cache miss.  The C++ mirror's
// gvh_deliver_blocks runs this schedule (C1 steady blocks 1.54 -> 2.50M tx/s,
// tests/test_block_paths.py::test_pipelined_replay_equals_block_by_block).
//
//	for h := range blocks {
//		app.BeginBlock(...)
//		if h == 0 {
//			app.PreVerifyTxs(blocks[0])
//		}
//		wait := func() {}
//		if h+1 < len(blocks) {
//			wait = app.PreVerifyAhead(blocks[h], blocks[h+1])
//		}
//		for _, tx := range blocks[h] {
//			app.DeliverTx(abci.RequestDeliverTx{Tx: tx})
//		}
//		app.EndBlock(...)
//		app.Commit()
//		wait()
//	}
func (app *BaseApp) PreVerifyAhead(cur, next [][]byte) (wait func()) {
	nop := func() {}
	if app.preVerifierAhead == nil || len(next) == 0 || app.deliverState == nil {
		return nop
	}
	verify := app.preVerifierAhead(app.deliverState.ctx, app.decodeAll(cur), app.decodeAll(next))
	if verify == nil {
		return nop
	}
	done := make(chan struct{})
	go func() {
		defer close(done)
		verify() // touches no state: the job's own account copies, the cache, the GPU
	}()
	return func() { <-done }
}

// prepareCheckTxs runs the state stage against the check state (the caller
// holds whatever serialises it with CheckTx / Commit); nil if nothing to do.
func (app *BaseApp) prepareCheckTxs(txs [][]byte) func() {
	if app.preVerifier == nil || len(txs) == 0 || app.checkState == nil {
		return nil
	}
	return app.preVerifier(app.checkState.ctx, app.decodeAll(txs))
}

// PreVerifyCheckTxs pre-verifies mempool txs against the check state.
func (app *BaseApp) PreVerifyCheckTxs(txs [][]byte) {
	if verify := app.prepareCheckTxs(txs); verify != nil {
		verify()
	}
}

// ---------------------------------------------------------------- Ingress

// Ingress pre-verifies mempool txs where they arrive concurrently, ahead of
// ABCI.  Wire it as the node's application (proxy.NewLocalClientCreator(in)
// at server/start.go:173 instead of the bare app): its CheckTx, Commit and
// InitChain take the lock that serialises the ingress' state reads with the
// check state, and everything else is the embedded BaseApp.  Feed Submit from
// the RPC broadcast handlers / the mempool reactor (a tx that is never
// submitted is simply verified by the decorator in CheckTx).
//
// Batches close at MaxTxs or MaxWait after their first tx; the state stage
// runs under the lock (a few microseconds per tx), the GPU call does not, so
// a CheckTx never waits on a GPU batch.  Submit never blocks: when the queue
// is full the tx is dropped from pre-verification (a cache miss later).
type Ingress struct {
	*BaseApp
	MaxTxs  int
	MaxWait time.Duration

	stateMu sync.Mutex // the check state: CheckTx / Commit / InitChain vs the ingress' reads
	queue   chan []byte
	done    chan struct{}
	once    sync.Once
}

// NewIngress starts the ingress batcher (64 txs or 200 us per batch, a queue
// of 8192 txs).
func NewIngress(app *BaseApp) *Ingress {
	in := &Ingress{BaseApp: app, MaxTxs: 64, MaxWait: 200 * time.Microsecond,
		queue: make(chan []byte, 8192), done: make(chan struct{})}
	go in.loop()
	return in
}

// Submit queues a tx for pre-verification (non-blocking).
func (in *Ingress) Submit(tx []byte) {
	select {
	case in.queue <- tx:
	default:
	}
}

// Close stops the batcher (idempotent).
func (in *Ingress) Close() { in.once.Do(func() { close(in.done) }) }

func (in *Ingress) loop() {
	for {
		var batch [][]byte
		select {
		case <-in.done:
			return
		case tx := <-in.queue:
			batch = append(batch, tx)
		}
		deadline := time.NewTimer(in.MaxWait)
	fill:
		for len(batch) < in.MaxTxs {
			select {
			case tx := <-in.queue:
				batch = append(batch, tx)
			case <-deadline.C:
				break fill
			case <-in.done:
				deadline.Stop()
				return
			}
		}
		deadline.Stop()
		in.stateMu.Lock()
		verify := in.BaseApp.prepareCheckTxs(batch)
		in.stateMu.Unlock()
		if verify != nil {
			verify() // sign bytes + GPU batch + cache fill: no lock held
		}
	}
}

// CheckTx implements abci.Application: BaseApp.CheckTx under the state lock.
func (in *Ingress) CheckTx(req abci.RequestCheckTx) abci.ResponseCheckTx {
	in.stateMu.Lock()
	defer in.stateMu.Unlock()
	return in.BaseApp.CheckTx(req)
}

// Commit implements abci.Application (it replaces the check state).
func (in *Ingress) Commit() abci.ResponseCommit {
	in.stateMu.Lock()
	defer in.stateMu.Unlock()
	return in.BaseApp.Commit()
}

// InitChain implements abci.Application (it creates the check state).
func (in *Ingress) InitChain(req abci.RequestInitChain) abci.ResponseInitChain {
	in.stateMu.Lock()
	defer in.stateMu.Unlock()
	return in.BaseApp.InitChain(req)
}

// ---------------------------------------------------------- CheckTxWindow

// CheckTxWindow batches CheckTx calls that arrive concurrently: the first
// request of a window opens it, later ones join, and the window closes when
// it holds MaxTxs requests or MaxWait after it opened; its txs are
// pre-verified in one batch, then every request runs the normal CheckTx
// (serialised: BaseApp.CheckTx is not re-entrant).  ReCheck requests skip
// signature verification (sigverify.go:172) and go straight through.
//
// Adaptive: a window only waits when requests are actually concurrent -- when
// another request is in flight, or the previous window held more than one.
// A lone request (every request under tendermint's serial delivery) flushes
// at once, so the window never adds latency there.
type CheckTxWindow struct {
	App     *BaseApp
	MaxTxs  int
	MaxWait time.Duration

	mu       sync.Mutex // guards cur, inflight, lastSize
	appMu    sync.Mutex // serialises App.CheckTx
	cur      *window
	inflight int // requests between join and the end of their CheckTx
	lastSize int // requests in the last flushed window
}

type window struct {
	txs  [][]byte
	done chan struct{}
	once sync.Once
}

// NewCheckTxWindow with the defaults of the C++ mirror (gvh_set_window): 64 txs, 200 us.
func NewCheckTxWindow(app *BaseApp) *CheckTxWindow {
	return &CheckTxWindow{App: app, MaxTxs: 64, MaxWait: 200 * time.Microsecond}
}

// CheckTx is BaseApp.CheckTx behind the accumulation window.
func (w *CheckTxWindow) CheckTx(req abci.RequestCheckTx) abci.ResponseCheckTx {
	if req.Type == abci.CheckTxType_Recheck {
		return w.checkTx(req)
	}
	b := w.join(req.Tx)
	<-b.done
	res := w.checkTx(req)
	w.mu.Lock()
	w.inflight--
	w.mu.Unlock()
	return res
}

func (w *CheckTxWindow) checkTx(req abci.RequestCheckTx) abci.ResponseCheckTx {
	w.appMu.Lock()
	defer w.appMu.Unlock()
	return w.App.CheckTx(req)
}

func (w *CheckTxWindow) join(tx []byte) *window {
	w.mu.Lock()
	lone := w.cur == nil && w.inflight == 0 && w.lastSize <= 1
	w.inflight++
	b := w.cur
	if b == nil {
		b = &window{done: make(chan struct{})}
		w.cur = b
		if !lone && w.MaxWait > 0 {
			time.AfterFunc(w.MaxWait, func() { w.flush(b) })
		}
	}
	b.txs = append(b.txs, tx)
	full := lone || w.MaxWait <= 0 || len(b.txs) >= w.MaxTxs
	w.mu.Unlock()
	if full {
		w.flush(b)
	}
	return b
}

func (w *CheckTxWindow) flush(b *window) {
	b.once.Do(func() {
		w.mu.Lock()
		if w.cur == b {
			w.cur = nil // later requests open a new window
		}
		txs := b.txs
		w.lastSize = len(txs)
		w.mu.Unlock()
		w.appMu.Lock() // the check state must not move under the pre-verifier's reads
		verify := w.App.prepareCheckTxs(txs)
		w.appMu.Unlock()
		if verify != nil {
			verify()
		}
		close(b.done)
	})
}
