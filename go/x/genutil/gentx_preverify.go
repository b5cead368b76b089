package genutil

// The genesis pre-verification hook (SURVEY.md §8f-1): DeliverGenTxs
// (x/genutil/gentx.go:96-114) delivers every gentx through the ante handler,
// one signature check per gentx.  This replacement encodes all gentxs first
// and hands their bytes to the pre-verifier in ONE batch (the app's
// baseapp.PreVerifyTxs, which predicts height-0 sign bytes -- account number
// 0, stdtx.go:249-253 -- and fills the verdict cache), then delivers them
// exactly as before, so the ante handler finds every verdict cached.
//
// Patch: delete DeliverGenTxs at x/genutil/gentx.go:96-114 and add this file;
// wire the hook at app construction (simapp/app.go, after SetPreVerifier):
//
//	genutil.SetGenTxPreVerifier(app.PreVerifyTxs)
//
// Behaviour is unchanged: same deliveries in the same order, the same panic
// on a failing gentx.  A malformed gentx JSON now panics before the first
// delivery instead of after the ones before it -- InitChain aborts either way
// with the same message.  Without a hook (nil) nothing is pre-verified.
//
// Source-level only here (no Go toolchain in the build image); the C++ mirror
// gvh_deliver_gentxs (host/gvhost.cpp) does the same and is tested
// (tests/test_block_paths.py).

import (
	"encoding/json"

	abci "github.com/tendermint/tendermint/abci/types"

	"github.com/cosmos/cosmos-sdk/codec"
	sdk "github.com/cosmos/cosmos-sdk/types"
	authtypes "github.com/cosmos/cosmos-sdk/x/auth/types"
	"github.com/cosmos/cosmos-sdk/x/genutil/types"
)

var genTxPreVerifier func(txs [][]byte)

// SetGenTxPreVerifier installs the hook DeliverGenTxs calls with every
// encoded gentx before the first is delivered (nil: none).
func SetGenTxPreVerifier(f func(txs [][]byte)) { genTxPreVerifier = f }

type deliverTxfn func(abci.RequestDeliverTx) abci.ResponseDeliverTx

// DeliverGenTxs decodes every genesis tx into a StdTx, pre-verifies the
// batch, then delivers each with deliverTx; it returns the staking module's
// ApplyAndReturnValidatorSetUpdates.
func DeliverGenTxs(
	ctx sdk.Context, cdc *codec.Codec, genTxs []json.RawMessage,
	stakingKeeper types.StakingKeeper, deliverTx deliverTxfn,
) []abci.ValidatorUpdate {
	encoded := make([][]byte, len(genTxs))
	for i, genTx := range genTxs {
		var tx authtypes.StdTx
		cdc.MustUnmarshalJSON(genTx, &tx)
		encoded[i] = cdc.MustMarshalBinaryBare(tx)
	}
	if genTxPreVerifier != nil && len(encoded) > 0 {
		genTxPreVerifier(encoded) // one batch: the signatures of every gentx
	}
	for _, bz := range encoded {
		if res := deliverTx(abci.RequestDeliverTx{Tx: bz}); !res.IsOK() {
			panic(res.Log)
		}
	}
	return stakingKeeper.ApplyAndReturnValidatorSetUpdates(ctx)
}
