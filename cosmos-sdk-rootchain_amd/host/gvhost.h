/*
 * gvhost.h -- C ABI of libgvhost.so: the host-side mirror (C++) of the
 * reference's signature-verification ante path and of the baseapp batching
 * hooks around it, built on libgpuverify.
 *
 * The reference is Go (no toolchain in this image), so the layer above the
 * GPU C-ABI is written in C++ and mirrors the reference with the same names,
 * argument meaning, gas accounting and error (codespace, code, log) results:
 *
 *   DefaultTxDecoder            x/auth/types/stdtx.go:321-338 (amino binary StdTx; bank MsgSend /
 *                               MsgMultiSend are the registered msgs, x/bank/types/codec.go:26-27)
 *   ValidateMemoDecorator       x/auth/ante/basic.go:61-77 (memo length + params gas)
 *   ConsumeTxSizeGasDecorator   x/auth/ante/basic.go:98-148
 *   SetPubKeyDecorator          x/auth/ante/sigverify.go:50-99
 *   ValidateSigCountDecorator   x/auth/ante/sigverify.go:265-294 (+ CountSubKeys stdtx.go:125-137)
 *   SigGasConsumeDecorator      x/auth/ante/sigverify.go:101-153, DefaultSigVerificationGasConsumer :299-322,
 *                               ConsumeMultisignatureVerificationGas :325-338
 *   BatchSigVerificationDecorator  replaces SigVerificationDecorator (sigverify.go:160-216): all leaves of
 *                               a tx (multisig fanned out, tendermint multisig.VerifyBytes semantics) are
 *                               answered from the verdict cache or verified in ONE libgpuverify batch;
 *                               failures are reported in signer order
 *   DeductFeeDecorator          x/auth/ante/fee.go:84-108 (the fee payer's account read)
 *   IncrementSequenceDecorator  x/auth/ante/sigverify.go:218-259
 *   SetGasMeter                 x/auth/ante/setup.go:67-76 (limit = the tx's fee gas; infinite at height 0)
 *   PreVerifyTxs                baseapp batching hook: one GPU batch for a block of txs,
 *                               sign bytes predicted with per-signer sequence prediction, verdicts cached
 *                               under SHA256(pub || sig || SHA256(signBytes)) in a bounded table
 *   DeliverBlock                the DeliverTx loop of a block (baseapp/abci.go:203-221) after PreVerifyTxs
 *   CheckTx window              CheckTx (baseapp/abci.go:165-196) through an accumulation window: calls
 *                               arriving within max_wait_us (or until max_txs) share one GPU batch
 *   DeliverGenTxs               x/genutil/gentx.go:96-114 (height 0: account number 0, infinite gas)
 *
 * Transactions are the amino binary StdTx bytes a node receives (DeliverTx /
 * CheckTx req.Tx).  A tx that does not decode gets code 2 (ErrTxDecode).
 *
 * No CPU fallback: every secp256k1 leaf goes to gv_verify_digests and every
 * ed25519 multisig sub-key leaf to gv_verify_ed25519_msgs (one batch each per
 * resolve); if a GPU batch fails the decorator returns GVH_EDEVICE and the
 * caller (the Go shim) re-verifies with the reference VerifyBytes (fail
 * closed).
 */
#ifndef GVHOST_H
#define GVHOST_H
#include <stddef.h>
#include <stdint.h>
#include "../../include/gpuverify.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GVH_OK 0
#define GVH_EINVAL -1
#define GVH_EDEVICE -2     /* the GPU batch failed: caller must fall back (fail closed) */
#define GVH_ENOVERIFIER -3 /* no gv_ctx attached and a secp256k1 leaf needed verifying */

typedef struct gvh_app gvh_app;

typedef struct gvh_result {
  uint32_t code;          /* 0 = OK, else the sdk error code (2 tx decode, 4 unauthorized, 8 invalid pubkey, ...) */
  char codespace[16];     /* "sdk" or "undefined" (panic) */
  char log[512];          /* sdkerrors.Wrap(...).Error() text */
  uint64_t gas_used;      /* gas consumed by the decorators that ran */
  uint32_t gpu_leaves;    /* secp256k1 leaves sent to the GPU for this tx */
  uint32_t cache_hits;    /* leaves answered by the verdict cache */
  uint64_t gas_wanted;    /* the tx's fee gas (0 if it did not decode) */
} gvh_result;

typedef struct gvh_stats {
  uint64_t gpu_calls;     /* libgpuverify batches issued */
  uint64_t gpu_leaves;    /* secp256k1 leaves verified on the GPU */
  uint64_t cache_hits, cache_misses;
  uint64_t memo_hits;     /* ante runs that reused PreVerifyTxs' decode + sign bytes */
  uint64_t windows;       /* CheckTx windows flushed */
  uint64_t window_txs;    /* txs that went through a window */
  uint64_t cache_entries, cache_capacity;
  uint64_t preverify_ns;  /* DeliverBlock: time in PreVerifyTxs (decode + plans + GPU) */
  uint64_t gpu_ns;        /* time in the GPU batches of PreVerifyTxs */
  uint64_t deliver_loop_ns; /* DeliverBlock: time in the serial ante loop */
} gvh_stats;

/* gpu may be NULL (then secp256k1 verification returns GVH_ENOVERIFIER). */
gvh_app* gvh_app_new(gv_ctx* gpu);
void gvh_app_free(gvh_app* app);

/* x/auth params (params.go:16-20 defaults: 7, 1000, 590). */
void gvh_set_params(gvh_app* app, uint64_t tx_sig_limit, uint64_t sig_cost_secp256k1, uint64_t sig_cost_ed25519);
/* Gas model.  kv_gas = 1 (default): the chain charges what the reference's
 * decorators charge besides signature gas -- every gas-metered account read
 * and write (gaskv, store/gaskv/store.go:36-52: 1000 + 3/byte read, 2000 +
 * 30/byte write of the proto account value), the five params reads of each
 * AccountKeeper.GetParams, and ConsumeTxSizeGas (10 per tx byte); reads happen
 * where the reference makes them, so a tx that fails at signer i is charged
 * the reads of signers 0..i only.  A nonzero fee's bank transfer is not
 * modelled (no balances).  kv_gas = 0: signature gas only. */
void gvh_set_gas_model(gvh_app* app, int kv_gas);
/* sdk.Context pieces the decorators read: chain id, block height (0 = genesis:
 * account number 0 in sign bytes, infinite gas), ReCheckTx flag.  gas_limit
 * 0 = SetGasMeter semantics (the tx's fee gas); nonzero overrides it. */
void gvh_set_context(gvh_app* app, const char* chain_id, int64_t height, int recheck, uint64_t gas_limit);

/* In-memory AccountKeeper.  pub_amino may be NULL/0 (pubkey not set). */
int gvh_set_account(gvh_app* app, const uint8_t addr20[20], uint64_t account_number, uint64_t sequence,
                    const uint8_t* pub_amino, size_t pub_len);
/* returns 1 if found; pub_amino_out (>= 512 bytes) may be NULL */
int gvh_get_account(gvh_app* app, const uint8_t addr20[20], uint64_t* account_number, uint64_t* sequence,
                    uint8_t* pub_amino_out, size_t* pub_len);

/* SetUpContext (gas meter) -> SetPubKey -> ValidateSigCount -> SigGasConsume ->
 * BatchSigVerification -> IncrementSequence on one amino StdTx.  Returns
 * GVH_OK when the chain ran (the tx verdict is in out->code), or a negative
 * GVH_E* infrastructure error. */
int gvh_ante(gvh_app* app, const uint8_t* tx, size_t tx_len, int simulate, gvh_result* out);

/* PreVerifyTxs: decode a block of txs, predict every signer's sign bytes
 * (sequence = state + earlier txs of the same signer here), verify the cache
 * misses in ONE GPU batch and fill the verdict cache; the decode and sign
 * bytes are memoised for the ante runs that follow.  No app lock is held
 * during the GPU call.  *n_leaves = secp256k1 leaves verified on the GPU. */
int gvh_preverify(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, size_t* n_leaves);
/* A block: PreVerifyTxs, then the ante chain of every tx in order (the
 * DeliverTx loop); out[i] is tx i's result. */
int gvh_deliver_block(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, gvh_result* out);
/* Same, returning only each tx's code (codes[i]; 0 = OK). */
int gvh_deliver_block_codes(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens,
                            uint32_t* codes);
/* n_blocks consecutive blocks (block_ntx[b] txs each, concatenated in txs /
 * lens / codes) delivered in order -- the results and final state of calling
 * gvh_deliver_block_codes once per block -- pipelined for block sync /
 * replay: block b+1 is pre-verified (its sequence prediction carrying block
 * b's increments and SetPubKeys) and its GPU batch runs while block b's
 * DeliverTx loop runs. */
int gvh_deliver_blocks(gvh_app* app, size_t n_blocks, const size_t* block_ntx, const uint8_t* const* txs,
                       const size_t* lens, uint32_t* codes);
/* genutil.DeliverGenTxs: the block path at height 0 (account number 0,
 * infinite gas); *first_failed = index of the first tx whose result is not OK
 * (the reference panics on it), or ntx if all passed. */
int gvh_deliver_gentxs(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, gvh_result* out,
                       size_t* first_failed);

/* CheckTx through the accumulation window: thread-safe and blocking; calls
 * arriving while a window is open share ONE PreVerifyTxs batch, flushed when
 * it holds max_txs txs or max_wait_us after its first tx; then each call runs
 * its own ante chain on the cached verdicts.  Defaults: 64 txs, 200 us.
 * Adaptive: a call opens a window only when calls are concurrent (another
 * call in flight, or the previous window held more than one); a lone call --
 * every call under tendermint's serial CheckTx delivery -- runs its ante
 * chain at once (its leaves in their own GPU batch) and waits for nothing.
 * max_wait_us = 0: never wait. */
int gvh_checktx(gvh_app* app, const uint8_t* tx, size_t tx_len, gvh_result* out);
void gvh_set_window(gvh_app* app, size_t max_txs, int64_t max_wait_us);

/* DefaultSigVerificationGasConsumer (x/auth/ante/sigverify.go:299-322) on its
 * own: pub_amino NULL/0 = nil pubkey. */
int gvh_consume_sig_gas(gvh_app* app, const uint8_t* sig, size_t sig_len, const uint8_t* pub_amino, size_t pub_len,
                        uint64_t gas_limit, gvh_result* out);

/* Verdict cache: bounded (CLOCK eviction in 8-way buckets), default 1<<20 entries. */
void gvh_cache_clear(gvh_app* app);
size_t gvh_cache_size(gvh_app* app);
void gvh_set_cache_capacity(gvh_app* app, size_t entries);
/* Host threads for PreVerifyTxs' decode / sign-bytes / SHA-256 stages
 * (default min(16, hardware threads)). */
void gvh_set_threads(gvh_app* app, int threads);
/* keyed = 1 (default): secp256k1 leaves verified through the GPU context's
 * key arena (gv_verify_digests_keyed); keys not yet resident are loaded
 * (gv_keys_load, once per distinct key) by batches of at least load_min
 * leaves (default 4096: blocks), and a smaller batch with an unknown key
 * takes the pub33 path.  keyed = 0: pub33 batches (gv_verify_digests).  Same
 * verdicts either way.  While keyed, the app owns the context's key arena
 * (a gv_keys_reset elsewhere is detected by gv_keys_generation). */
void gvh_set_keyed(gvh_app* app, int keyed, size_t load_min);
/* gpu_hash = 1: PreVerifyTxs of a block being delivered, with an empty
 * verdict cache, hands the secp256k1 leaves' sign bytes to the GPU
 * (gv_verify_msgs / gv_verify_msgs_keyed, SHA-256 in the batch) instead of
 * hashing them on the host; 0 (default; env GVH_GPU_HASH): host SHA-256 +
 * gv_verify_digests*, measured faster.  Same verdicts either way. */
void gvh_set_gpu_hash(gvh_app* app, int on);
int gvh_get_gpu_hash(gvh_app* app);
/* The keyed-path policy in force (defaults: 1, GV_KEY_LOAD_MIN, GV_KEY_CAP of gpuverify.h). */
void gvh_get_keyed(gvh_app* app, int* keyed, size_t* load_min, size_t* key_cap);
void gvh_get_stats(gvh_app* app, gvh_stats* out);

/* StdSignBytes (x/auth/types/stdtx.go:292-312): canonical JSON.  Returns the
 * length; writes at most cap bytes. */
size_t gvh_std_sign_bytes(const char* chain_id, uint64_t account_number, uint64_t sequence,
                          const char* fee_json, const char* const* msgs_json, size_t n_msgs,
                          const char* memo, uint8_t* out, size_t cap);
/* DefaultTxDecoder + StdTx.GetSignBytes for one amino StdTx: writes the sign
 * bytes (at most cap) and returns their length; a tx that does not decode
 * returns 0 and writes the decode error text (NUL-terminated, at most
 * err_cap bytes) into err. */
size_t gvh_tx_sign_bytes(const uint8_t* tx, size_t tx_len, const char* chain_id, uint64_t account_number,
                         uint64_t sequence, uint8_t* out, size_t cap, char* err, size_t err_cap);
/* crypto.PubKey.Address() of an amino pubkey: secp256k1 RIPEMD160(SHA256(pub33)),
 * multisig SHA256(amino bytes)[:20], ed25519 SHA256(pub32)[:20]. 0 = ok. */

/* ---- IBC 07-tendermint light-client commit checks ----
 * tendermint v0.33.4 types/validator_set.go VerifyCommit (lite2 Verify ->
 * VerifyAdjacent / VerifyNonAdjacent from x/ibc/07-tendermint/update.go:88)
 * and VerifyCommitTrusting (VerifyNonAdjacent, misbehaviour.go:88-97) for n
 * commits: every signature their loops could read is verified in ONE
 * gv_verify_ed25519_msgs batch, each loop then walked in reference order over
 * the verdicts -- same code, index and tallies as the sequential loop.  The
 * caller supplies what needs the tendermint types: verifyCommitBasic's
 * verdict and each signature's VoteSignBytes(chainID, i). */
#define GVH_COMMIT_FLAG_ABSENT 1   /* types.BlockIDFlagAbsent */
#define GVH_COMMIT_FLAG_COMMIT 2   /* types.BlockIDFlagCommit (counts toward the tally) */
#define GVH_COMMIT_FLAG_NIL 3      /* types.BlockIDFlagNil (verified, not tallied) */
typedef struct gvh_commit {
  int trusting;                  /* 0: VerifyCommit (signature i <-> validator i); 1: VerifyCommitTrusting */
  int64_t trust_num, trust_den;  /* trusting: tmmath.Fraction (lite.DefaultTrustLevel = 1/3) */
  int basic_ok;                  /* verifyCommitBasic(commit, height, blockID) == nil */
  size_t n_vals;
  const uint8_t* val_pub32;      /* validator ed25519 keys (32 bytes each) */
  const uint8_t* val_addr20;     /* validator addresses (trusting) */
  const int64_t* val_power;      /* voting powers */
  size_t n_sigs;
  const uint8_t* flag;           /* BlockIDFlag per signature */
  const uint8_t* sig_addr20;     /* CommitSig.ValidatorAddress (trusting) */
  const uint8_t* sig64;          /* signatures, 64-byte stride */
  const uint32_t* sig_len;       /* their lengths (!= 64: VerifyBytes is false) */
  const uint8_t* msg_blob;       /* VoteSignBytes(chainID, i) at msg_off[i], msg_len[i] */
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  int keys_trusted;              /* the set is already trusted (the trusted next validators of
                                    VerifyCommitTrusting, or an adjacent header's set matching the
                                    trusted NextValidatorsHash): its keys may be loaded into the
                                    ed25519 key arena.  0: a relayer-supplied set -- verified without
                                    loading its keys, so fresh sets cannot churn the arena */
} gvh_commit;
#define GVH_COMMIT_OK 0
#define GVH_COMMIT_BASIC 1         /* verifyCommitBasic's error (the caller's) */
#define GVH_COMMIT_SIZE 2          /* NewErrInvalidCommitSignatures(vals.Size(), len(commit.Signatures)) */
#define GVH_COMMIT_WRONG_SIG 3     /* "wrong signature (#idx): %X" */
#define GVH_COMMIT_NOT_ENOUGH 4    /* ErrNotEnoughVotingPowerSigned{Got: got, Needed: needed} */
#define GVH_COMMIT_DOUBLE_VOTE 5   /* "double vote from %v (idx and idx2)" */
#define GVH_COMMIT_BAD_TRUST 6     /* trust level outside [1/3, 1]: the reference panics */
typedef struct gvh_commit_result {
  int32_t code, idx, idx2;
  int64_t got, needed;           /* the tally when the loop ended and the power needed */
} gvh_commit_result;
int gvh_verify_commits(gvh_app* app, size_t n, const gvh_commit* commits, gvh_commit_result* out);

int gvh_pubkey_address(const uint8_t* pub_amino, size_t len, uint8_t out20[20]);
/* sdk.AccAddress.String(): bech32 "cosmos1..." (types/address.go:222-234). */
size_t gvh_bech32_address(const uint8_t addr20[20], char* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
