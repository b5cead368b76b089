package baseapp

// PreVerifyTxs and the CheckTx accumulation window (SURVEY.md §8f-1): the
// block / mempool batching hooks that fill the signature verdict cache the
// BatchSigVerificationDecorator reads (go/x/auth/ante/batch_sigverify.go).
//
// ABCI v0.33 hands the app one tx per DeliverTx / CheckTx
// (baseapp/abci.go:165-221), so a batch is formed before them:
//   - a block: the executor calls PreVerifyTxs(block.Txs) after BeginBlock,
//     before its DeliverTx loop;
//   - genesis: genutil.DeliverGenTxs (x/genutil/gentx.go:96-114) calls it on
//     the marshalled gentxs before delivering them;
//   - the mempool: CheckTxWindow gathers concurrent CheckTx requests into one
//     batch (size or deadline), pre-verifies it, then runs each CheckTx.
// Nothing here changes a verdict: a missing or mispredicted cache entry is a
// miss and the decorator verifies it itself.
//
// One field is added to the BaseApp struct (baseapp/baseapp.go:45-92):
//
//	preVerifier PreVerifier // fills the signature verdict cache (SetPreVerifier)
//
// Source-level only in this repository (no Go toolchain in the build image).

import (
	"sync"
	"time"

	abci "github.com/tendermint/tendermint/abci/types"

	sdk "github.com/cosmos/cosmos-sdk/types"
)

// PreVerifier fills the verdict cache for a batch of decoded txs against the
// state of ctx (x/auth/ante.NewPreVerifier).
type PreVerifier func(ctx sdk.Context, txs []sdk.Tx)

// SetPreVerifier registers the pre-verification hook (app construction,
// simapp/app.go:335-339, next to SetAnteHandler).
func (app *BaseApp) SetPreVerifier(pv PreVerifier) {
	if app.sealed {
		panic("SetPreVerifier() on sealed BaseApp")
	}
	app.preVerifier = pv
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
	app.preVerifier(st.ctx, app.decodeAll(txs))
}

// PreVerifyCheckTxs pre-verifies mempool txs against the check state.
func (app *BaseApp) PreVerifyCheckTxs(txs [][]byte) {
	if app.preVerifier == nil || len(txs) == 0 || app.checkState == nil {
		return
	}
	app.preVerifier(app.checkState.ctx, app.decodeAll(txs))
}

// CheckTxWindow gathers concurrent CheckTx requests: the first request of a
// window opens it, the window closes when it holds MaxTxs requests or MaxWait
// after it opened, its txs are pre-verified in one batch, and then every
// request runs the normal CheckTx (serialised: BaseApp.CheckTx is not
// re-entrant).  ReCheck requests skip signature verification
// (sigverify.go:172) and go straight through.
type CheckTxWindow struct {
	App     *BaseApp
	MaxTxs  int
	MaxWait time.Duration

	mu    sync.Mutex // guards cur
	appMu sync.Mutex // serialises App.CheckTx
	cur   *window
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
	return w.checkTx(req)
}

func (w *CheckTxWindow) checkTx(req abci.RequestCheckTx) abci.ResponseCheckTx {
	w.appMu.Lock()
	defer w.appMu.Unlock()
	return w.App.CheckTx(req)
}

func (w *CheckTxWindow) join(tx []byte) *window {
	w.mu.Lock()
	b := w.cur
	if b == nil {
		b = &window{done: make(chan struct{})}
		w.cur = b
		time.AfterFunc(w.MaxWait, func() { w.flush(b) })
	}
	b.txs = append(b.txs, tx)
	full := len(b.txs) >= w.MaxTxs
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
		w.mu.Unlock()
		w.appMu.Lock() // the check state must not move under the pre-verifier
		w.App.PreVerifyCheckTxs(txs)
		w.appMu.Unlock()
		close(b.done)
	})
}
