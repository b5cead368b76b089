/*
 * gvhost.h -- C ABI of libgvhost.so: the host-side mirror (C++) of the
 * reference's signature-verification ante path, built on libgpuverify.
 *
 * The reference is Go (no toolchain in this image), so the layer above the
 * GPU C-ABI is written in C++ and mirrors the reference's decorators with the
 * same names, argument meaning, gas accounting and error (codespace, code,
 * log) results:
 *
 *   SetPubKeyDecorator          x/auth/ante/sigverify.go:50-99
 *   ValidateSigCountDecorator   x/auth/ante/sigverify.go:265-294 (+ CountSubKeys stdtx.go:125-137)
 *   SigGasConsumeDecorator      x/auth/ante/sigverify.go:101-153, DefaultSigVerificationGasConsumer :299-322,
 *                               ConsumeMultisignatureVerificationGas :325-338
 *   BatchSigVerificationDecorator  replaces SigVerificationDecorator (sigverify.go:160-216): all leaves of
 *                               a tx (multisig fanned out, tendermint multisig.VerifyBytes semantics) are
 *                               verified in ONE libgpuverify batch; failures are reported in signer order
 *   IncrementSequenceDecorator  x/auth/ante/sigverify.go:218-259
 *   PreVerifyTxs                baseapp batching hook: one GPU batch for a block of txs,
 *                               sign bytes predicted with per-signer sequence prediction, verdicts cached
 *                               under (pub33 || sig64 || SHA256(signBytes))
 *
 * Transactions are passed in a flat encoding (the decoded StdTx the Go shim
 * would hold -- amino tx decoding is out of scope, SURVEY.md §2 "Codec"):
 *   u32 n_msgs, { u32 len, msg sign-bytes JSON (canonical, Msg.GetSignBytes) }
 *   u32 len, fee JSON (StdFee.Bytes(), canonical)
 *   u32 len, memo (UTF-8)
 *   u32 n_signers, { 20-byte address }            (tx.GetSigners() order)
 *   u32 n_sigs,    { u32 len, amino pubkey bytes; u32 len, signature bytes }
 * All integers little-endian.
 *
 * No CPU fallback for secp256k1: if the GPU batch fails the decorator
 * returns GVH_EDEVICE and the caller (the Go shim) re-verifies with the
 * reference VerifyBytes.  ed25519 multisig leaves are verified on the CPU
 * (OpenSSL), as in the reference.
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
  uint32_t code;          /* 0 = OK, else the sdk error code (4 unauthorized, 8 invalid pubkey, ...) */
  char codespace[16];     /* "sdk" or "undefined" (panic) */
  char log[512];          /* sdkerrors.Wrap(...).Error() text */
  uint64_t gas_used;      /* gas consumed by the decorators that ran */
  uint32_t gpu_leaves;    /* secp256k1 leaves sent to the GPU for this tx */
  uint32_t cache_hits;    /* leaves answered by the verdict cache */
} gvh_result;

/* gpu may be NULL (then secp256k1 verification returns GVH_ENOVERIFIER). */
gvh_app* gvh_app_new(gv_ctx* gpu);
void gvh_app_free(gvh_app* app);

/* x/auth params (params.go:16-20 defaults: 7, 1000, 590). */
void gvh_set_params(gvh_app* app, uint64_t tx_sig_limit, uint64_t sig_cost_secp256k1, uint64_t sig_cost_ed25519);
/* sdk.Context pieces the decorators read: chain id, block height (0 = genesis:
 * account number 0 in sign bytes), ReCheckTx flag, gas limit (0 = infinite). */
void gvh_set_context(gvh_app* app, const char* chain_id, int64_t height, int recheck, uint64_t gas_limit);

/* In-memory AccountKeeper.  pub_amino may be NULL/0 (pubkey not set). */
int gvh_set_account(gvh_app* app, const uint8_t addr20[20], uint64_t account_number, uint64_t sequence,
                    const uint8_t* pub_amino, size_t pub_len);
/* returns 1 if found; pub_amino_out (>= 512 bytes) may be NULL */
int gvh_get_account(gvh_app* app, const uint8_t addr20[20], uint64_t* account_number, uint64_t* sequence,
                    uint8_t* pub_amino_out, size_t* pub_len);

/* SetPubKey -> ValidateSigCount -> SigGasConsume -> BatchSigVerification ->
 * IncrementSequence on one tx.  Returns GVH_OK when the chain ran (the tx
 * verdict is in out->code), or a negative GVH_E* infrastructure error. */
int gvh_ante(gvh_app* app, const uint8_t* tx, size_t tx_len, int simulate, gvh_result* out);

/* Pre-verify a block of txs in one GPU batch and fill the verdict cache.
 * Sequences are predicted as state sequence + earlier txs of the same signer
 * in this call.  *n_leaves = secp256k1 leaves verified. */
int gvh_preverify(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, size_t* n_leaves);
/* DefaultSigVerificationGasConsumer (x/auth/ante/sigverify.go:299-322) on its
 * own: pub_amino NULL/0 = nil pubkey. */
int gvh_consume_sig_gas(gvh_app* app, const uint8_t* sig, size_t sig_len, const uint8_t* pub_amino, size_t pub_len,
                        uint64_t gas_limit, gvh_result* out);
void gvh_cache_clear(gvh_app* app);
/* Host threads for PreVerifyTxs' decode / sign-bytes / SHA-256 stages
 * (default min(4, hardware threads)). */
void gvh_set_threads(gvh_app* app, int threads);
size_t gvh_cache_size(gvh_app* app);

/* StdSignBytes (x/auth/types/stdtx.go:292-312): canonical JSON.  Returns the
 * length; writes at most cap bytes. */
size_t gvh_std_sign_bytes(const char* chain_id, uint64_t account_number, uint64_t sequence,
                          const char* fee_json, const char* const* msgs_json, size_t n_msgs,
                          const char* memo, uint8_t* out, size_t cap);
/* crypto.PubKey.Address() of an amino pubkey: secp256k1 RIPEMD160(SHA256(pub33)),
 * multisig SHA256(amino bytes)[:20], ed25519 SHA256(pub32)[:20]. 0 = ok. */
int gvh_pubkey_address(const uint8_t* pub_amino, size_t len, uint8_t out20[20]);
/* sdk.AccAddress.String(): bech32 "cosmos1..." (types/address.go:222-234). */
size_t gvh_bech32_address(const uint8_t addr20[20], char* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
