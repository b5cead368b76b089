/*
 * gpuverify.h -- C ABI of libgpuverify.so, the MI355X (gfx950) batched
 * secp256k1 transaction-signature verifier.
 *
 * Drop-in boundary.  Every entry point below replaces, for a
 * whole batch at once, the reference's per-signature call
 *
 *     pubKey.VerifyBytes(signBytes, sig)            x/auth/ante/sigverify.go:210
 *
 * i.e. tendermint v0.33.4 crypto/secp256k1 PubKeySecp256k1.VerifyBytes
 * (secp256k1_nocgo.go), reached through SigVerificationDecorator.AnteHandle
 * (x/auth/ante/sigverify.go:170-216) and, for multisig leaves, through
 * multisig.PubKeyMultisigThreshold.VerifyBytes (the type switch at
 * x/auth/ante/sigverify.go:303-321 names both key types).  out_ok[i] is
 * exactly VerifyBytes(msg_i, sig_i) for pubkey pub33_i: 1 = true, 0 = false.
 * Cryptographic rejection is never an error code.
 *
 * Plain pointers and sizes only (cgo / ctypes / JNI friendly).  The caller owns
 * every buffer; the library copies inputs into its own device memory and keeps
 * no caller pointer after a call returns (the gv_submit_* calls excepted: they
 * keep theirs until gv_wait).  Host-buffer gv_verify_* calls are synchronous
 * and a gv_ctx may be shared by concurrent threads (calls on one device
 * serialise; every use of a device's scratch, on any stream, is ordered after
 * the previous one, so gv_dev_* calls on different caller streams never
 * overwrite each other's in-flight inputs).
 * INTEGRATION.md shows the Go (cgo) binding a maintainer adds as
 * crypto/gpuverify and the BatchSigVerificationDecorator built on it.
 */
#ifndef GPUVERIFY_H
#define GPUVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes: 0 = OK, negative = infrastructure error.  On any nonzero
 * return the caller must not use out_ok and should re-verify on the CPU
 * (fail-closed; SURVEY.md §5 "Failure detection"). */
#define GV_OK        0
#define GV_EINVAL   -1   /* bad argument (null pointer, misaligned device ptr, ...) */
#define GV_ENODEV   -2   /* no usable HIP device / bad device id */
#define GV_EHIP     -3   /* HIP runtime or kernel error */
#define GV_ENOMEM   -4   /* device or host allocation failed */
#define GV_EFAULT   -5   /* injected fault (option "fault_inject") */

typedef struct gv_ctx gv_ctx;

/* Open a context on dev_ids[0..n_dev) (HIP ordinals); n_dev == 0 -> every
 * visible device.  Builds the per-device G table.  Replaces nothing in the
 * reference (which has no device state); the Go shim calls it once at app
 * construction (simapp/app.go:335-339 wiring site). */
int gv_open(const int* dev_ids, int n_dev, gv_ctx** out);
void gv_close(gv_ctx* ctx);
int gv_num_devices(const gv_ctx* ctx);

/* Batch VerifyBytes over messages.  Item i: pubkey pub33 + 33*i (SEC1
 * compressed, as stored by secp256k1.PubKeySecp256k1 [33]byte), signature
 * sig64 + 64*i (R||S big-endian, tendermint's 64-byte format), message
 * msg_blob[msg_off[i] .. msg_off[i] + msg_len[i]) (StdSignBytes,
 * x/auth/types/stdtx.go:248-259).  Signatures whose length is not 64 are
 * decided (false) by the caller before the call, exactly like VerifyBytes'
 * first check.  Replaces the loop body at x/auth/ante/sigverify.go:194-213. */
int gv_verify_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                   const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                   uint8_t* out_ok);

/* Same with the messages already hashed: dig32 + 32*i = SHA256(msg_i)
 * (tendermint crypto.Sha256).  This is VerifyBytes minus its hashing step
 * (btcec Signature.Verify(hash, pub) preceded by the tendermint checks). */
int gv_verify_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                      const uint8_t* dig32, uint8_t* out_ok);

/* Packed-bitmap variants: bit (i % 64) of out_bits[i / 64] is item i's
 * verdict; ceil(n/64) words are written (unused high bits 0). */
int gv_verify_digests_bits(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                           const uint8_t* dig32, uint64_t* out_bits);
int gv_verify_msgs_bits(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                        const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                        uint64_t* out_bits);

/* Device-resident entry points for callers whose batch already lives in HBM
 * (benchmarks, a node that stages blocks on the GPU).  dev_slot indexes the
 * context's devices; d_* are device pointers on that device (4-byte aligned);
 * d_bits receives ceil(n/64) words; stream is a hipStream_t (NULL = the
 * context's stream).  Asynchronous: results are ready when the stream is. */
int gv_dev_verify_digests(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub33,
                          const void* d_sig64, const void* d_dig32, void* d_bits, void* stream);
int gv_dev_verify_msgs(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub33,
                       const void* d_sig64, const void* d_msg_blob, const void* d_msg_off,
                       const void* d_msg_len, void* d_bits, void* stream);

/* Device memory and stream helpers for callers of the gv_dev_* entry points
 * that have no HIP runtime of their own (bench.py, tests).  kind: 1 = host to
 * device, 2 = device to host, 3 = device to device; copies are ordered on the
 * context stream of dev_slot and synchronous. */
int gv_dev_alloc(gv_ctx* ctx, int dev_slot, size_t bytes, void** d_ptr);
int gv_dev_free(gv_ctx* ctx, int dev_slot, void* d_ptr);
int gv_dev_copy(gv_ctx* ctx, int dev_slot, void* dst, const void* src, size_t bytes, int kind);
int gv_dev_sync(gv_ctx* ctx, int dev_slot);
/* A non-blocking HIP stream on dev_slot for the gv_dev_* calls' `stream`
 * argument (callers without a HIP runtime of their own), its synchronisation
 * and destruction. */
int gv_dev_stream_create(gv_ctx* ctx, int dev_slot, void** stream_out);
int gv_dev_stream_sync(gv_ctx* ctx, int dev_slot, void* stream);
int gv_dev_stream_destroy(gv_ctx* ctx, int dev_slot, void* stream);

/* Account pubkey cache.  The reference amino-decodes and
 * btcec-parses an account's pubkey on every VerifyBytes
 * (x/auth/types/account.go:65-72 -> secp256k1_nocgo.go ParsePubKey), and a
 * node verifies the same accounts block after block.  gv_keys_load parses n
 * SEC1 keys once (prefix, x < p, square root) and keeps each key's table of
 * 16 multiples resident in HBM on every device of the context (1,280 B per
 * key, plus the tables of 2^35 Q, 2^70 Q, 2^100 Q for the small-batch keyed
 * kernels: 5.4 KB per key) and, with option "keys_k6" (default), the
 * throughput ladder's 11 tables of 32 multiples of 2^(12 k) Q on one Z (28 KB
 * per key: 1M accounts = 34 GB of the 288 GB); slot_out[i] receives key i's
 * slot.
 * A key that ParsePubKey rejects gets a slot too, and every verify against it
 * is false.  Slots are assigned in load order and stay valid until
 * gv_keys_reset.  Loading must not race keyed verifies of the same context. */
int gv_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub33, uint32_t* slot_out);
int gv_keys_reset(gv_ctx* ctx);
size_t gv_keys_count(const gv_ctx* ctx);
/* Number of gv_keys_reset calls on ctx so far: a caller that keeps a
 * pubkey -> slot map drops it when the generation moved (slots of an older
 * generation may name other keys). */
uint64_t gv_keys_generation(const gv_ctx* ctx);

/* Routing policy shared by the callers above this ABI (the Go shim
 * go/crypto/gpuverify reads these through cgo; the C++ mirror host/gvhost.cpp
 * uses them as its defaults), so the two cannot drift apart:
 *   GV_CPU_CROSSOVER  batches smaller than this go to the reference CPU
 *                     VerifyBytes (one host core answers a
 *                     single signature in ~0.20 ms, the sliced small-batch
 *                     kernels ~0.21 ms at any size up to 256);
 *   GV_KEY_LOAD_MIN   only batches of at least this many leaves (a block)
 *                     load keys that are not resident yet; a smaller batch
 *                     (CheckTx) goes keyed only when all its keys are
 *                     resident, else pub33 (loading per
 *                     CheckTx window cost 35.8k -> 5.1k tx/s);
 *   GV_KEY_CAP        arena size at which the caller resets the arena
 *                     (5.4 KB of HBM per key). */
#define GV_CPU_CROSSOVER 4
#define GV_KEY_LOAD_MIN 4096
#define GV_KEY_CAP (1u << 22)
/* ... and the ed25519 key arena's (gv_ed_keys_load: 72 KB of HBM per key). */
#define GV_ED_KEY_CAP (1u << 16)

/* Key-arena readback (tests, tools): for each slot, the affine point the
 * arena holds for it, out_xy64 + 64*i = x || y (32 bytes each, big-endian),
 * and out_ok[i] = its ParsePubKey verdict (a slot >= gv_keys_count(): zeros
 * and 0).  Reads the first device's arena. */
int gv_keys_point(gv_ctx* ctx, size_t n, const uint32_t* slots, uint8_t* out_xy64, uint8_t* out_ok);

/* VerifyBytes with the key given by slot: out_ok[i] is exactly what
 * gv_verify_digests / gv_verify_msgs return with pub33 = the key loaded into
 * slot[i]; a slot >= gv_keys_count() gives false.  Same batching, errors and
 * multi-device split as the pub33 entry points; batches up to "lat_max" take
 * the fused small-batch kernel with the key's table read from the arena. */
int gv_verify_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                            const uint8_t* dig32, uint8_t* out_ok);
int gv_verify_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                         const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                         uint8_t* out_ok);
/* Device-resident keyed digests: d_slot = n u32 slots on dev_slot. */
int gv_dev_verify_digests_keyed(gv_ctx* ctx, int dev_slot, size_t n, const void* d_slot, const void* d_sig64,
                                const void* d_dig32, void* d_bits, void* stream);

/* ---- ed25519 ------------------------------------------
 * out_ok[i] = tendermint v0.33.4 PubKeyEd25519(pub32[i]).VerifyBytes(msg_i,
 * sig64[i]) for a 64-byte signature, i.e. go1.14 crypto/ed25519 Verify:
 * sig[63] & 224 == 0, S < L (ScMinimal), A = FromBytes(pub) (non-canonical y
 * accepted, no small-order check), encode([S]B - [SHA-512(R||A||M) mod L]A)
 * == R as bytes.  Replaces, for a batch, the per-leaf call reached through
 * multisig.PubKeyMultisigThreshold.VerifyBytes for ed25519 sub-keys
 * (x/auth/ante/sigverify.go:210 via :303-306 / :325-338).  Signatures of any
 * other length are false without a call (VerifyBytes' first check), as for
 * secp256k1.  msg_blob may be NULL when every length is 0. */
int gv_verify_ed25519_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub32, const uint8_t* sig64,
                           const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                           uint8_t* out_ok);
/* Device-resident: d_pub32 (n x 32) and d_sig64 (n x 64) 16-byte aligned,
 * d_msg_off u64 / d_msg_len u32 per item; accept bitmap into d_bits
 * (ceil(n/64) u64 words).  Asynchronous on `stream` (NULL: the library's). */
int gv_dev_verify_ed25519_msgs(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub32, const void* d_sig64,
                               const void* d_msg_blob, const void* d_msg_off, const void* d_msg_len, void* d_bits,
                               void* stream);
/* Cached ed25519 keys: the IBC 07-tendermint light client verifies a
 * validator set's commit signatures block after block
 * (x/ibc/07-tendermint/update.go:88 lite.Verify, misbehaviour.go:88-97
 * VerifyCommitTrusting), and multisig accounts keep their ed25519 sub-keys.
 * gv_ed_keys_load runs FromBytes once per key and keeps the comb table of -A
 * (j * 16^w * (-A), w < 64, j <= 8: 72 KB per key) and the raw key bytes
 * resident on every device; slot_out[i] receives key i's slot (a key
 * FromBytes rejects gets one too, and every verify against it is false).
 * gv_verify_ed25519_msgs_keyed gives exactly gv_verify_ed25519_msgs's verdict
 * with pub32 = the key loaded into slot[i] (a slot >= gv_ed_keys_count()
 * gives false).  Batches up to "ed_lat_max" (default 2048) take k_ed_lat_sl
 * (one signature per block, no doublings: ~0.1 ms end to end), larger ones the
 * throughput kernels.  Loading must not race keyed verifies of the same
 * context; gv_ed_keys_generation counts gv_ed_keys_reset calls. */
int gv_ed_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub32, uint32_t* slot_out);
int gv_ed_keys_reset(gv_ctx* ctx);
size_t gv_ed_keys_count(const gv_ctx* ctx);
uint64_t gv_ed_keys_generation(const gv_ctx* ctx);
int gv_verify_ed25519_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                                 const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                                 uint8_t* out_ok);

/* Options: "max_batch" (lanes per device launch, default 1<<20, at most
 * 0xFFFFFF00),
 * "lat_max" (batches of at most this many items -- per device slice -- take
 * a fused small-batch kernel, default 8192; 0 = never),
 * "lat_sl_max" (batches of at most this many items take the limb-sliced
 * small-batch kernels k_verify_lat_sl / k_verify_lat16_sl, one signature per
 * block; larger ones up to lat_max the four-lanes-per-signature
 * k_verify_lat / k_verify_lat16; default 2048),
 * "lat_max_keyed" / "lat_sl_max_keyed" (the same two bounds for keyed
 * batches, defaults 14336 / 1536: the sliced keyed kernel takes four waves
 * per signature, and the 16-lanes-per-signature keyed kernel beats the keyed
 * pipeline to ~14k; setting "lat_max" / "lat_sl_max" sets these too),
 * "lat_sliced" (0/1: 0 never takes the sliced kernels; default 1),
 * "ed_unc_lat_max" (uncached ed25519 host batches of at most this many
 * items take k_ed_lat_unc: one signature per block, FromBytes(A) in the
 * kernel; default 2048, 0 = never),
 * "lat_rows_max" (pub33 sliced batches of at most this many items take
 * k_verify_lat_sl4: five waves per signature, each ladder wave's four rows on
 * one accumulator, G from the k6 tables after the ladder; default 512, 0 =
 * never, env GV_LAT_ROWS_MAX),
 * "lat_zero_copy" (0/1: host-buffer digest batches on the sliced kernels
 * are read by the kernel straight from the pinned staging buffer and answered
 * as verdict bytes in pinned memory -- no H2D, memset or D2H; default 1),
 * "pipe_chunk" (host-buffer calls past lat_max: first chunk of the two-stream
 * copy/compute pipeline per device, default 262144; 0 = one chunk per
 * max_batch), "pipe_growth" (each later chunk at most this many times the one
 * before, default 4: the staging of chunk i+1 hides under the kernels of
 * chunk i), "stage_threads" (pageable -> pinned staging copy threads PER
 * DEVICE, the slice's own thread included: each device stages through its own
 * pool; default half the process's CPUs -- affinity capped by the cgroup
 * quota -- split over the devices, 1..8 each),
 * "stage_pieces" (pageable host chunks of at least 65,536 items are staged
 * into pinned memory in this many pieces, each piece's H2D right behind its
 * copy; default 2, env GV_STAGE_PIECES),
 * "lat_kw" (0/1: keyed sliced small batches whose slots all have the
 * resident arena's one-window wide tables take k_verify_lat16_kw -- no
 * doublings -- instead of the kn tables' k_verify_lat16_kn; default 1, env
 * GV_LAT_KW),
 * "async_chunk" / "async_growth" (submitted batches staged through the
 * library -- pageable buffers, messages: fixed chunks of async_chunk items,
 * each later one at most async_growth times the one before; default 262144
 * and 1, env GV_ASYNC_CHUNK / GV_ASYNC_GROWTH), "async_whole" (0/1:
 * submitted digest batches read in place from gv_host_alloc memory run as
 * ONE chunk when they queue behind a batch still in flight -- their copies
 * and front kernels then run under the previous batch's ladder -- and take
 * the pipe_chunk ramp on an idle device; default 1, env GV_ASYNC_WHOLE),
 * "h2d_serial" (0/1: a host slice's chunks send their inputs one after the
 * other -- each chunk's H2D waits for the previous chunk's -- so the chunk
 * the GPU needs first is not slowed by the next one's transfer; default 1,
 * env GV_H2D_SERIAL),
 * "gfull_item" (0/1: the per-item pub33 route -- batches not grouped by
 * key -- also adds G on the unsplit u1 from the "gfull" tables: 11 G
 * additions instead of 14; default 1, env GV_GFULL_ITEM),
 * "inv_small" (0/1: batches under 2^19 items fold fewer signatures per lane
 * in the s^-1 batch inversion, so it stays short where it precedes the first
 * ladder -- a host slice's first chunk; default 1, env GV_INV_SMALL),
 * "slice_plain_first" (host-buffer pub33 slices grouped by key: this many
 * items first on the per-item pipeline while the slice's key tables build;
 * 0 = off, the default; env GV_SLICE_PLAIN_FIRST),
 * "group_keys" (0/1: a pub33 batch past the small-batch bound with at least
 * "group_min" items (default 16384) whose distinct keys number at most
 * items / "group_div" (default 5) parses each distinct key once -- grouped
 * on the device, tables built into a per-batch arena, the items verified by
 * the keyed pipeline; same verdicts; default 1, env GV_GROUP_KEYS),
 * "ed_group" (0/1: ed25519 throughput batches -- gv_verify_ed25519_msgs and
 * the device-resident variant -- of at least "ed_group_min" items (default
 * 196608; host chunks of 262,144 qualify) with at most items / 16 (and 16384) distinct keys build each key's
 * comb table once (k_ed_keys into a per-batch arena) and verify on k_ed_keyed,
 * lanes in slot order; same verdicts; default 1, env GV_ED_GROUP),
 * "ed_keyed" (0/1: gv_verify_ed25519_msgs_keyed batches past "ed_lat_max"
 * run one signature per lane against the cached comb tables of -A -- 64
 * table adds for [h](-A), no doublings, lanes in slot order; 0 = the
 * throughput kernels over the slots' raw keys; same verdicts; default 1, env
 * GV_ED_KEYED),
 * "ed_group_r64" (0/1: the grouped route's per-batch ed25519 key tables are
 * radix-64 combs -- 43 windows of 32 entries, 43 additions per [h](-A)
 * instead of 64; same verdicts; default 1, env GV_ED_GROUP_R64),
 * "ed_btab16" (0/1: k_ed_keyed -- cached keys past "ed_lat_max" and grouped
 * keys -- and the per-item throughput kernels add [s]B from a radix-2^16 comb table of B, j * 65536^w * B for
 * w < 16 and j <= 2^15 (56.6 MB per device, built on first use): 16
 * additions instead of 32; same verdicts; default 1, env GV_ED_BTAB16),
 * "sort_keys" (0/1: keyed throughput batches on the 4-group ladder -- cached
 * slots, grouped keys -- run their lanes in slot order: a counting sort by
 * slot, the signature rows read in that order, the accept bits gathered back
 * to item order; same verdicts; default 1, env GV_SORT_KEYS),
 * "pipeline_dev" (0/1: device-resident calls on the context stream past the
 * small-batch bound are pipelined -- consecutive calls alternate scratch sets,
 * their unpack / s^-1 / prep kernels run under the previous call's ladder on
 * a stream above the ladders' priority (env GV_LADDER_PRIO "front", the
 * default; "ladder" / "equal" for A/B); a caller stream is never pipelined;
 * default 1, env GV_PIPELINE),
 * "two_ladders" (0/1: pipelined calls' ladders alternate two streams, so the
 * next ladder fills the current one's tail; bitmap writes stay in call order;
 * default 1, env GV_TWO_LADDERS),
 * "gfull" (0/1: keyed batches on the 4-group ladder add G from the unsplit
 * u1 = e/s -- 11 signed 25-bit windows from tables of 2^o G (6 GiB per device,
 * built by gv_open) -- instead of 14 GLV windows; same verdicts;
 * default 1, env GV_GFULL; route counter GV_ROUTE_K4F),
 * "k6" (0/1: in-batch grouped keys on the 6-bit-window ladder -- 4 groups of
 * 32-entry key tables, 30 doublings, G from 11 24-bit windows of the unsplit
 * u1 (5.5 GiB of tables, built by gv_open); same verdicts; default 0, env
 * GV_K6; route counter GV_ROUTE_K6),
 * "kg" (0 or 6 / 7 / 9: in-batch grouped keys on the many-group 5-bit
 * ladder -- k4's 16-entry tables of 5-bit windows split over kg groups
 * instead of 4, so the ladder runs ceil(26 / kg) positions (kg 7: 15
 * doublings, 9: 10) for kg x 16 table entries per key; G from 11 24-bit
 * windows of the unsplit u1 after the last doubling, on the real curve; same
 * verdicts; takes precedence over "k6"; env GV_KG; route counter
 * GV_ROUTE_KG),
 * "keys_k6" (0/1: gv_keys_load also builds each key's 6-bit-window tables --
 * 11 groups of 32 entries on one Z, 28 KB per key beside the 5.4 KB of k4
 * tables -- and keyed throughput batches whose slots all have them run the
 * 6-doubling ladder; small keyed batches keep the k4 tables; same verdicts;
 * default 1, env GV_KEYS_K6; route counter GV_ROUTE_KN),
 * "keys_wide" (0/1/2: gv_keys_load also builds each key's 9-bit-window
 * tables of 256 entries on one Z -- 2 (default): one window per group, 15
 * tables (240 KB per key), no doublings and 30 Q additions per verify; 1: two
 * windows per group, 8 tables (128 KB), 9 doublings -- in an arena of their
 * own that grows by doubling while the HBM budget holds it and the device
 * keeps room for the k4 / k6 arena to reach key_cap; with 2, an arena that no
 * longer fits moves to the two-window layout (the loaded keys are read back
 * from the k4 tables and rebuilt); keyed throughput batches whose slots all
 * have them run that ladder (else the k6 one); same verdicts; the layout of
 * an arena is chosen when it starts from slot 0; env GV_KEYS_WIDE; route
 * counters GV_ROUTE_KW / GV_ROUTE_KW2),
 * "key_cap" / "ed_key_cap" (the callers' reset points of the secp256k1 /
 * ed25519 key arenas: an arena grows by doubling up to it and exactly past it;
 * defaults GV_KEY_CAP / GV_ED_KEY_CAP, env of the same names; the Go shim sets
 * both to its KeyCap / EdKeyCap at Open),
 * "hbm_budget_mb" (MiB of optional device tables per device -- the G tables
 * past the GLV pair, the key arenas, the grouping arenas; a table past the
 * budget is not built and batches take the schedule that needs less, with the
 * same verdicts: k6 -> k4 -> the 125-doubling keyed ladder, full-scalar G ->
 * GLV G; keys_load returns GV_ENOMEM when not even the k4 arena fits; 0 = no
 * limit, the default; env GV_HBM_BUDGET_MB; the large G tables are built by
 * gv_open unless env GV_EAGER_TABLES=0),
 * "time_kernels" (0/1: record HIP events around each kernel stage; the
 * ladder's time is its own start to end),
 * "fault_inject" (0/1: every verify call fails with GV_EFAULT; test hook). */
int gv_set_option(gv_ctx* ctx, const char* key, long long val);
/* The current value of a schedule option set by gv_set_option or its
 * environment variable: "kg", "k6", "gfull", "keys_k6", "keys_wide",
 * "group_keys", "sort_keys", "pipeline_dev", "two_ladders", "key_cap",
 * "max_batch", "async_chunk", "async_growth", "async_whole", and (read
 * only) "kw_qw", the resident arena's wide-window width this library was
 * built with.  GV_EINVAL for any other key.  Instrumentation (bench route
 * attribution). */
int gv_get_option(gv_ctx* ctx, const char* key, long long* val);

/* Asynchronous host batches.  gv_submit_* queue a batch with the arguments
 * of the matching gv_verify_* entry point and return at once with a ticket;
 * gv_wait(ticket) blocks until that batch's verdicts are in out_ok and
 * returns its result (the gv_verify_* codes; a ticket is waited for once).
 * Batches run in submission order per context, each device's slices as one
 * stream of chunks: the next batch's staging, key grouping and key tables run
 * while the previous batch's last chunks compute, so a caller that keeps a
 * batch queued ahead (the next block's PreVerifyTxs, a replay) gets the
 * device-resident pipeline's overlap from host buffers.  Unlike gv_verify_*,
 * the library keeps the caller's pointers until gv_wait returns: the buffers
 * (ideally gv_host_alloc memory, read in place) must stay valid and unchanged
 * until then.  gv_wait is also a ticket's release: a caller that abandons a
 * batch (an error of its own between submit and wait) still waits for it,
 * since the library reads and writes its buffers until the batch is done; a
 * ticket never waited keeps a few hundred bytes of bookkeeping until gv_close,
 * which finishes the queued batches and frees it.  gv_keys_load /
 * gv_keys_reset wait for every submitted batch first, and submissions made
 * while one of them runs wait until it returns.  Replaces nothing in the
 * reference (its ante handler verifies synchronously, x/auth/ante/
 * sigverify.go:210); it is how baseapp's pre-verification hook keeps the
 * GPU busy across blocks (baseapp/abci.go:203-221). */
int gv_submit_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
                      uint8_t* out_ok, uint64_t* ticket);
int gv_submit_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* dig32,
                            uint8_t* out_ok, uint64_t* ticket);
int gv_submit_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* msg_blob,
                   const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok, uint64_t* ticket);
int gv_submit_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* msg_blob,
                         const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok, uint64_t* ticket);
int gv_wait(gv_ctx* ctx, uint64_t ticket);

/* With "time_kernels" on: milliseconds of the last launch's stages on dev_slot
 * (unpack+sha, prep, ecmult), measured with HIP events on the launch stream. */
int gv_last_stage_ms(gv_ctx* ctx, int dev_slot, float* unpack_ms, float* prep_ms, float* ecmult_ms);

/* With "time_kernels" on: average stage milliseconds over every launch on
 * dev_slot since the previous call (at most the last 256 launches); *count
 * receives the number of launches averaged.  Synchronises dev_slot. */
int gv_stage_stats(gv_ctx* ctx, int dev_slot, int* count, double* unpack_ms, double* prep_ms,
                   double* ecmult_ms);

/* Same, per stage: ms[0] unpack (+ SHA-256 on the message path), ms[1]
 * k_scalar_inv, ms[2] k_prep, ms[3] k_ecmult (fused latency kernel: ms[3]). */
int gv_stage_stats4(gv_ctx* ctx, int dev_slot, int* count, double ms[4]);
/* Host-buffer calls on a multi-device context: per device slot, the wall time
 * (ms) and item count of that device's slice in the last gv_verify_* call
 * (bench.py --inproc: per-device rates).  Returns the number of slots written. */
int gv_last_slices(gv_ctx* ctx, double* ms_out, size_t* n_out, int cap);
/* Pinned host memory for a caller's input buffers: a host-buffer digest call
 * (gv_verify_digests[_bits|_keyed]) whose pub33 / slot, sig64 and dig32
 * arrays lie in such memory skips the library's pageable -> pinned staging
 * copy (the device reads them in place: DMA, or zero-copy for small batches).
 * The Go shim packs its batches into these buffers. */
int gv_host_alloc(gv_ctx* ctx, size_t bytes, void** out);
int gv_host_free(gv_ctx* ctx, void* p);
/* In-batch key grouping (options "group_keys", "ed_group"): on dev_slot, the
 * number of batches -- secp256k1 and ed25519 -- that took the grouped (keyed)
 * pipeline and the distinct keys whose tables they built. */
int gv_group_stats(gv_ctx* ctx, int dev_slot, uint64_t* batches, uint64_t* keys);
/* Batches per secp256k1 schedule on dev_slot since gv_open, out[GV_ROUTES]:
 * GV_ROUTE_PUB33 (per-item pipeline: k_prep + k_ecmult), GV_ROUTE_KEYED125
 * (keyed, 125-doubling ladder), GV_ROUTE_K4 (keyed 4-group ladder over the
 * key arena), GV_ROUTE_K6 (in-batch key grouping on the 6-bit-window ladder),
 * GV_ROUTE_LAT (small pub33 batches: gv_lat.hip kernels), GV_ROUTE_LAT_KEYED
 * (small keyed batches), GV_ROUTE_K4F (the 4-group ladder with the G half on
 * the unsplit scalar, 25-bit windows), GV_ROUTE_ITEMF (the per-item pipeline
 * with the G half on the unsplit scalar, "gfull_item"), GV_ROUTE_KN (keyed
 * batches on the resident arena's k6 tables: 11 groups of 6-bit windows, 6
 * doublings, option "keys_k6"), GV_ROUTE_ED_LAT (small uncached ed25519
 * host batches on k_ed_lat_unc, option "ed_unc_lat_max"), GV_ROUTE_KW (keyed
 * batches on the resident arena's wide-window tables, one 9-bit window per
 * group: 15 groups, no doublings, option "keys_wide"), GV_ROUTE_KW2 (the same
 * with two windows per group: 8 groups, 9 doublings), GV_ROUTE_KG (in-batch
 * key grouping on the many-group 5-bit ladder, option "kg").  Instrumentation only (bench route
 * attribution, node metrics). */
#define GV_ROUTE_PUB33 0
#define GV_ROUTE_KEYED125 1
#define GV_ROUTE_K4 2
#define GV_ROUTE_K6 3
#define GV_ROUTE_LAT 4
#define GV_ROUTE_LAT_KEYED 5
#define GV_ROUTE_K4F 6
#define GV_ROUTE_ITEMF 7
#define GV_ROUTE_KN 8
#define GV_ROUTE_ED_LAT 9
#define GV_ROUTE_KW 10
#define GV_ROUTE_KW2 11
#define GV_ROUTE_KG 12
#define GV_ROUTES 13
int gv_route_stats(gv_ctx* ctx, int dev_slot, uint64_t out[GV_ROUTES]);

const char* gv_strerror(int code);

/* Test hook: run one arithmetic building block per item on dev_slot
 * (op codes in gv_kernels.hip k_debug; in/out = n x 16 little-endian u32
 * host arrays).  Used by the GPU unit tests only. */
int gv_debug_op(gv_ctx* ctx, int dev_slot, int op, size_t n, const uint32_t* in, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* GPUVERIFY_H */
