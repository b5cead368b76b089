// gv_kernels.h -- internal interface between the C-ABI runtime (gv_runtime.cpp)
// and the HIP kernels (gv_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef GV_GW
#define GV_GW 20                // G / lambda*G signed window width (bits); multiple of GV_QW
#endif
#define GV_QW 5                 // Q / lambda*Q signed window width (bits)
#define GV_GTAB_N (1 << (GV_GW - 1))   // multiples 1..2^(GV_GW-1) per table (64 B each)
#define GV_GSTEP (GV_GW / GV_QW)       // Q windows per G window
#define GV_QTAB_N 16            // multiples 1..2^(GV_QW-1) of Q per lane
#define GV_QENT_WORDS 20        // Q-table entry: x[9], y[9] raw 29-bit limbs + 2 pad words (80 B)
#define GV_QTAB_WORDS (GV_QTAB_N * GV_QENT_WORDS + (GV_QTAB_N - 1) * 9)  // per lane: entries (AoS) + Z-ratio rows (SoA)
#define GV_QWIN 26              // Q windows over a 128-bit GLV half: positions 0,5,..,125
#define GV_GWIN ((GV_QWIN - 1) / GV_GSTEP + 1)   // G windows at positions 0, GV_GW, ..
#define GV_DIGIT_ROWS (GV_QWIN + 2 * GV_GWIN)    // Q: packed int16 pair per window; G: int32 per digit
#ifndef GV_INV_M
#define GV_INV_M 32             // signatures folded per lane by k_scalar_inv (A/B: profiles/r03/invm_ab)
#endif

static_assert(GV_GW % GV_QW == 0, "G windows must sit on Q window positions");
static_assert(GV_GW * GV_GWIN >= 130 && GV_GW * (GV_GWIN - 1) <= GV_QW * (GV_QWIN - 1), "G window count");

#ifdef __cplusplus
extern "C" {
#endif

// Key-ordered lanes scratch (gv_sort.hip), all device memory.
typedef struct gvk_sort {
  uint32_t *cnt, *off;          // kcount + 1 bucket counts / exclusive offsets
  uint32_t *pos, *perm;         // item -> lane, lane -> item (C words each)
  uint32_t* kslot;              // slot per lane (C words)
  uint64_t* bits;               // slot-ordered accept bits (C / 64 words)
  void* temp;                   // scan scratch (gvk_sort_temp_bytes)
  size_t temp_bytes;
} gvk_sort;

// One device batch of C lanes (C % 256 == 0, n <= C live items).  All pointers
// are device pointers.  Either dig32 (digest path) or msg_* (message path).
typedef struct gvk_batch {
  uint32_t n, C;
  const uint8_t* pub33;
  const uint8_t* sig64;
  const uint8_t* dig32;
  const uint8_t* msg_blob;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  const uint32_t* gtab;         // 2 tables (G, lambda*G) x GV_GTAB_N entries x 16 words, AoS
  uint32_t *in_x, *in_pfx, *in_r, *in_s, *in_e;
  uint32_t *digits;             // GV_DIGIT_ROWS rows: packed Booth digits per window (16 rows reused as scratch)
  uint32_t *zq, *flags, *qtab;  // shared Z of the Q table (8 rows), flags, Q table (192 rows)
  uint64_t* bits;               // C/64 words, bit (i%64) of word i/64
  hipEvent_t ev[4];             // optional: after unpack/sha, after scalar_inv, after prep, after ecmult
  hipEvent_t ev_ecm_start;      // optional: the ladder kernel's start (after any wait on st_ecm)
  // Pipelined calls (st_ecm set): the front kernels (unpack, s^-1, prep) run on
  // the launch stream, the ladder on st_ecm after ecm_ready -- consecutive
  // batches' front kernels then fill the previous ladder's tail.
  hipStream_t st_ecm;
  hipEvent_t ecm_ready;
  // Consecutive pipelined calls may run their ladders on two streams (the
  // next ladder fills the current one's tail): the call's final bitmap write
  // (k_unsort_bits, or the ladder itself when unsorted) waits on bits_wait
  // (the previous call's) and records bits_done, so results land in call order.
  hipEvent_t bits_wait, bits_done;
  int unpacked;                 // the SoA rows are already written (in-batch key grouping ran k_unpack)
  uint32_t inv_m;               // k_scalar_inv signatures per lane (0: gvk_inv_m(C))
  hipEvent_t keys_ready;        // optional: the batch's key tables are built on another stream; k_prep waits
  // keyed batch (kslot != NULL, pub33 unused): item i's key is arena slot kslot[i]
  const uint32_t* kslot;        // n slots (device)
  const uint32_t* kqt;          // arena Q tables, row per slot (GV_QTAB_N x GV_QENT_WORDS words)
  const uint32_t* kzq;          // arena table Z: 8 rows of stride kC
  const uint32_t* kok;          // arena ParsePubKey verdicts
  uint32_t kC, kcount;          // arena capacity (row stride) and slots in use
  // keyed batches with gtab4 set take k_ecmult_k4 (30-doubling 4-group ladder)
  const uint32_t* kqt2;         // arena group tables (2^35 Q, 2^70 Q, 2^100 Q), on the slot's kzq
  const uint32_t* gtab4;        // GV_KEY2_TABLES x (G-type, lambda) tables of 2^35 G, 2^70 G, 2^100 G
  // k6 set: kqt / kqt2 hold 32-entry group tables of k6 groups (4: the grouped
  // route, k_keys_build_rows6; GV_KN_ARENA_NG: the resident arena; kqt2 rows
  // slot * (k6 - 1) + group - 1) and the ladder is k_ecmult_kn<k6> over gtab6
  // (GV_K6_GTAB_WORDS: the full-scalar 24-bit-window G tables); gtab4 unused
  const uint32_t* gtab6;
  int k6;
  // kqw == 1 (with k6 == GV_KW_NG1 or GV_KW_NG2): kqt / kqt2 / kzq are the
  // resident arena's wide-window tables (GV_KW_NT entries per group) and the
  // ladder is k_ecmult_kn<GV_KW_QW, k6>.  kqw == 2: the grouped route's
  // 5-bit many-group tables (GV_QTAB_N entries, k6 groups, one of GV_KG_NGS):
  // k_ecmult_kn<GV_QW, k6>
  int kqw;
  // k4 batches with gtabf set: the G half on the unsplit scalar (GV_GF_*),
  // k_prep<.., GF> digits and k_ecmult_k4<true> over gtabf (GV_GF_WORDS)
  const uint32_t* gtabf;
  // key-ordered lanes (gv_sort.hip; keyed k4 batches with srt.perm set): the
  // lanes run in slot order, the bits are gathered back to item order
  gvk_sort srt;
} gvk_batch;
// k_scalar_inv's fold for a batch of C lanes: GV_INV_M from 2^19 lanes up
// (the throughput pipeline: fewest instructions, the kernel runs beside a
// ladder); below, C / 65,536 (at least 4) so it still launches ~1,024 waves
// -- there it is latency-bound on the path to the first ladder (a host
// slice's first chunk), and its duration follows the per-lane chain length.
inline uint32_t gvk_inv_m(uint32_t C) {
  if (C >= (1u << 19)) return GV_INV_M;
  const uint32_t m = C / 65536u;
  return m < 4u ? 4u : m > (uint32_t)GV_INV_M ? (uint32_t)GV_INV_M : m;
}
// scan scratch bytes for nbuckets = kcount + 1 buckets
size_t gvk_sort_temp_bytes(uint32_t nbuckets);
// counting sort of n items by slot (clamped to kcount): pos / perm / kslot of so
hipError_t gvk_sort_slots(const gvk_sort* so, uint32_t n, const uint32_t* kslot, uint32_t kcount, hipStream_t st);
hipError_t gvk_unpack_perm(const uint8_t* sig64, const uint8_t* dig32, const uint32_t* perm, uint32_t n, uint32_t C,
                           uint32_t* r, uint32_t* s, uint32_t* e, hipStream_t st);
hipError_t gvk_unsort_bits(uint32_t n, const uint32_t* pos, const uint64_t* sbits, uint64_t* bits, hipStream_t st);

// Key arena row of one slot: Q table entries only (the Z-ratio scratch of the
// build lives in the batch scratch).
#define GV_KEY_WORDS (GV_QTAB_N * GV_QENT_WORDS)

// Keyed latency schedule (gv_lat.hip k_verify_lat16): the 26 five-bit windows
// of each 128-bit GLV half split into GV_LGRP groups starting at windows
// 0, 7, 14, 20 (bit offsets 0, 35, 70, 100).  The key arena holds, besides
// Q's table, the tables of 2^35 Q, 2^70 Q and 2^100 Q (rows of kqt2, Z in
// kzq2); glat holds the 16 multiples of 2^(5 w0) G and 2^(5 w0) lambda G
// per group (affine, 8 x 32 words x, y per entry).
#define GV_LGRP 4
#define GV_LAT16_SIGS 8                                   // signatures per 128-thread block: 16 lanes each
#define GV_KEY2_TABLES (GV_LGRP - 1)
#define GV_GLAT_WORDS (GV_LGRP * 2 * GV_QTAB_N * 16)

// The 6-bit-window keyed ladders (k_ecmult_kn<NG>): the key tables hold 32
// multiples per group (6-bit signed windows: 22 per 128-bit GLV half), the
// 22 windows split into NG groups -- the first R = 22 - (P - 1) NG groups of
// P = ceil(22 / NG) windows, the rest of P - 1 -- each with its own table of
// 2^(6 w0) Q on ONE shared Z, so the ladder runs P positions: 6 (P - 1)
// doublings and 44 Q additions.  NG = 4 ("k6": groups at windows 0, 6, 12,
// 17, 30 doublings; the grouped route's per-batch tables) and the resident
// arena's NG = GV_KN_ARENA_NG (more groups: fewer doublings per verify, more
// table memory per key, built once at gv_keys_load).  The lambda-Q entries go
// through the lambda frame (two beta products per position), and G is taken
// on the unsplit u1 = e/s: 11 signed 24-bit windows (window j at bit 24 j)
// added after the last doubling from 2^23-entry tables of 2^(24 j) G
// (5.5 GiB per device).  Group layout: gv_kernels.hip KLayout.
#define GV_K6_QW 6
#define GV_K6_NT 32                                       // table entries per group
#define GV_K6_QWIN 22
#ifndef GV_K6_GW
#define GV_K6_GW 24
#endif
#define GV_K6_GWIN ((257 + GV_K6_GW - 1) / GV_K6_GW)    // 11 windows at 24 bits
#define GV_K6_GNTAB GV_K6_GWIN                            // one G table per window
#define GV_K6_GTAB_N (1u << (GV_K6_GW - 1))
#define GV_K6_KEY_WORDS (GV_K6_NT * GV_QENT_WORDS)       // one group table (2,560 B)
#define GV_K6_GTAB_WORDS ((size_t)GV_K6_GNTAB * GV_K6_GTAB_N * 16)
#ifndef GV_KN_ARENA_NG
#define GV_KN_ARENA_NG 11                                 // resident arena: 11 groups of 2 windows, 6 doublings
#endif
static_assert(GV_K6_QWIN + GV_K6_GWIN <= GV_DIGIT_ROWS, "k6 digits fit the digit rows");
static_assert(GV_K6_QW * GV_K6_QWIN >= 130 && GV_K6_GW * GV_K6_GWIN >= 257, "k6 windows cover the scalars");

// The resident arena's wide-window tables (option "keys_wide",
// k_ecmult_kn<GV_KW_QW, NG>): 2^(QW-1) multiples per group, the signed QW-bit
// windows of each 128-bit GLV half one per group (NG = GV_KW_NG1: one ladder
// position, no doublings) or two per group (GV_KW_NG2: 2 positions).  QW = 11
// (default, round 6): 1,024 entries, 12 windows, 24 Q additions; 12 groups
// and no doublings (768 KiB of tables per key), or 6 groups and 11 doublings
// (384 KiB).  G as on the k6 ladders (11 24-bit windows after the last
// doubling, gtab6).  Built at gv_keys_load beside the k6 tables while the key
// set fits (kw2, then kn on the k6 tables otherwise).  A/B on one box,
// c2_key_cache (65,536 keys), one window per group: QW 7 / 8 / 9 =
// 329-344 / 366 / 380-381M/s (round 5, profiles/r05/kw/); round 6
// (profiles/r06/ab/kqw/): QW 9 / 10 / 11 / 12 = 421-430 / 452-467 / 482-488 /
// 500-505M/s, serialized ladder 2.12-2.16 / 1.90-1.95 / 1.82-1.84 /
// 1.71-1.74 ms; 12 doubles the tables again (1.5 MiB per key, 96 GiB for
// 65,536 keys) for +3.5 %, so 11 is the default and 12 an A/B build.
#ifndef GV_KW_QW
#define GV_KW_QW 11
#endif
#define GV_KW_NT (1 << (GV_KW_QW - 1))                    // 1,024 table entries per group
#define GV_KW_QWIN ((130 + GV_KW_QW - 1) / GV_KW_QW)      // 12 windows per GLV half
// Entry format: 16 = canonical words x[8] y[8] (64 B: a gather never
// straddles two cache lines, and 20 % less memory than the 80-B raw-limb
// entries, 20; 32 pads those to a line -- A/B builds).
#ifndef GV_KW_ENT_WORDS
#define GV_KW_ENT_WORDS 16
#endif
#define GV_KW_KEY_WORDS (GV_KW_NT * GV_KW_ENT_WORDS)     // one group table (65,536 B)
#define GV_KW_NG1 GV_KW_QWIN                              // one window per group: 12 groups
#define GV_KW_NG2 ((GV_KW_QWIN + 1) / 2)                  // two windows per group: 6 groups
static_assert(GV_KW_QW >= 7 && GV_KW_QW <= 12 && GV_KW_NG1 <= 19, "wide arena layout");
static_assert(GV_KW_QWIN + GV_K6_GWIN <= GV_DIGIT_ROWS, "wide-window digits fit the digit rows");
static_assert(GV_KW_QW * GV_KW_QWIN >= 130, "wide windows cover the GLV halves");

// The grouped route's many-group ladder (option "kg", k_ecmult_kn<GV_QW, NG>,
// round 6): the in-batch key tables keep k4's 16-entry 5-bit windows (26 per
// GLV half) but split them over NG groups instead of 4, so the ladder runs
// ceil(26 / NG) positions -- NG = 7: 15 doublings instead of 30, NG = 9: 10 --
// for NG x 16 table entries per key (k4: 64).  G as on the k6 ladders: 11
// signed 24-bit windows of the unsplit u1 after the last doubling from gtab6,
// on the real curve (one frame change, no per-entry lift).  NG must be one of
// GV_KG_NGS (the instantiated layouts); NG = 4 is k4's layout and tables
// (k_keys_tables) with G after the last doubling.
#define GV_KG_NGS 4, 6, 7, 9
#define GV_KG_MAXNG 9
static_assert(GV_QWIN + GV_K6_GWIN <= GV_DIGIT_ROWS, "kg digits fit the digit rows");

// The k4 ladder's G half on the unsplit scalar (k_ecmult_k4<true>): u1 = e/s
// is not GLV-split; its 11 signed 25-bit windows (window j at bit 25 j) are
// added from 2^24-entry tables of 2^o G for six offsets o (gv_kernels.hip
// kGFOff), window j at ladder position p reading the table of offset
// 25 j - 5 p.  11 G additions per verify instead of 14 and no lambda tables:
// 6 GiB per device.
#define GV_GF_W 25
#define GV_GF_WIN 11
#define GV_GF_NTAB 6
#define GV_GF_TAB_N (1u << (GV_GF_W - 1))
#define GV_GF_WORDS ((size_t)GV_GF_NTAB * GV_GF_TAB_N * 16)
static_assert(GV_QWIN + GV_GF_WIN <= GV_DIGIT_ROWS, "full-scalar G digits fit the digit rows");
static_assert(GV_GF_W * GV_GF_WIN >= 257, "the windows cover a 256-bit scalar plus the Booth carry");

// Small-batch latency path (gv_lat.hip): GV_LAT_SIGS signatures per block of
// 128 threads, one fused kernel (after k_sha256 on the message path).  bits
// receives ceil(n / GV_LAT_SIGS) 16-bit words (the caller zeroes the tail of
// the last 64-bit word).
#define GV_LAT_SIGS 16
typedef struct gvk_lat {
  uint32_t n, C;                // C: stride of e_soa rows (>= n)
  const uint8_t* pub33;
  const uint8_t* sig64;
  const uint8_t* dig32;
  const uint8_t* msg_blob;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  const uint32_t* gtab;
  uint32_t* e_soa;              // message path: 8 rows of C words
  uint64_t* bits;
  uint8_t* out8;                // sliced kernels: non-null -> one verdict byte per item here (e.g.
                                // mapped pinned host memory), bits unused and not zeroed
  hipEvent_t ev[1];             // optional: after the SHA stage
  // keyed batch (kslot != NULL, pub33 unused): tables from the key arena
  const uint32_t* kslot;
  const uint32_t* kqt;
  const uint32_t* kzq;
  const uint32_t* kok;
  uint32_t kC, kcount;
  // keyed batches take k_verify_lat16: the group tables below
  const uint32_t* kqt2;         // GV_KEY2_TABLES rows per slot (row slot * 3 + group - 1)
  const uint32_t* kzq2;         // GV_KEY2_TABLES x 8 rows of stride kC
  const uint32_t* glat;         // GV_GLAT_WORDS
  // pub33 sliced batches with gtab6 set (the runtime: n <= lat_rows_max)
  // take k_verify_lat_sl4 (row-parallel ladders, G from the 24-bit tables)
  const uint32_t* gtab6;
  // keyed sliced batches with kn != 0 (and gtab6): k_verify_lat16_kn over the
  // resident arena's kn tables (kqt = kqt6, kqt2 = kqt62, kzq = kzq6)
  int kn;
} gvk_lat;

// ed25519 (ed_verify.hip): one signature per lane over C lanes (C % 256 == 0).
#define GV_ED_ATAB_WORDS 324            // per-lane table j(-A), j = 0..8: 9 x 36 words, lane-major
#define GV_ED_ROWS (GV_ED_ATAB_WORDS + 9)  // + h (8 rows) + the prep verdict (1 row)
#define GV_ED_BTAB_WORDS (32 * 129 * 27)  // resident comb table j * 256^w * B
typedef struct gvk_ed {
  uint32_t n, C;
  const uint8_t* pub32;         // n x 32
  const uint8_t* sig64;         // n x 64
  const uint8_t* msg_blob;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  uint32_t* atab;               // scratch: C x GV_ED_ATAB_WORDS lane-major table, then h (8) + verdict SoA rows
  const uint32_t* btab;         // GV_ED_BTAB_WORDS
  const uint32_t* btab16;       // GV_ED_BTAB16_WORDS or null ([s]B in 16 additions instead of 32)
  uint64_t* bits;               // C/64 words
} gvk_ed;
hipError_t gvk_ed_btab(uint32_t* btab, hipStream_t st);
// The radix-2^16 comb table j * 65536^w * B, w < 16, j <= 2^15 (k_ed_keyed's [s]B).
#define GV_ED_BTAB16_WORDS ((size_t)16 * 32769 * 27)
hipError_t gvk_ed_btab16(uint32_t* btab16, hipStream_t st);
hipError_t gvk_ed_verify(const gvk_ed* b, hipStream_t st);
// ed25519 key arena (gv_ed_keys_load): per slot the comb table of -A,
// j * 16^w * (-A), w < 64, j = 1..8, cached form (36 words each), the raw key
// words (8) and the FromBytes verdict.
#define GV_EDK_WORDS (64 * 8 * 36)
// The grouped route's radix-64 comb tables: 43 windows of 32 entries per key.
#define GV_EDK64_WORDS (43 * 32 * 36)
typedef struct gvk_edl {
  uint32_t n;
  const uint32_t* slot;         // n key slots
  const uint8_t* sig64;         // n x 64
  const uint8_t* msg_blob;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  const uint32_t* ktab;         // kcap x GV_EDK_WORDS
  const uint32_t* kpub;         // kcap x 8
  const uint32_t* kok;          // kcap
  uint32_t kcount;
  const uint32_t* btab;         // GV_ED_BTAB_WORDS
  uint8_t* out8;                // n verdict bytes
  const uint8_t* pub32;         // gvk_ed_lat_unc: n x 32 key bytes (slot / ktab / kpub / kok unused)
} gvk_edl;
// wbase (may be null: one lane per key does everything): n * 64 * 36 words of
// scratch for the window bases -- the chain and the table adds then run as
// two launches (k_ed_keys_chain, k_ed_keys_tab), same table words.  rb: the
// comb radix bits, 4 (GV_EDK_WORDS per key) or 6 (GV_EDK64_WORDS; needs wbase).
hipError_t gvk_ed_keys(const uint8_t* pub32, uint32_t n, uint32_t base, uint32_t* ktab, uint32_t* kpub, uint32_t* kok,
                       uint32_t* wbase, int rb, hipStream_t st);
hipError_t gvk_ed_lat(const gvk_edl* b, hipStream_t st);
// Small ed25519 batches against uncached keys (k_ed_lat_unc): b->pub32 per item.
hipError_t gvk_ed_lat_unc(const gvk_edl* b, hipStream_t st);
// Large ed25519 batches against cached keys (k_ed_keyed): one signature per
// lane, lane g takes item perm[g] (null: g), verdict byte out8[item].
typedef struct gvk_edk {
  uint32_t n;
  const uint32_t* perm;         // n lanes -> items (gv_sort.hip), or null
  const uint32_t* slot;         // n key slots (item order)
  const uint8_t* sig64;         // n x 64
  const uint8_t* msg_blob;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  const uint32_t* ktab;
  const uint32_t* kpub;
  const uint32_t* kok;
  uint32_t kcount;
  const uint32_t* btab;
  const uint32_t* btab16;       // GV_ED_BTAB16_WORDS, or null: [s]B from btab (32 additions instead of 16)
  int rb;                       // ktab's comb radix bits: 4 (GV_EDK_WORDS per key; 0 = 4) or 6 (GV_EDK64_WORDS)
  uint8_t* out8;                // n verdict bytes (device)
} gvk_edk;
hipError_t gvk_ed_keyed(const gvk_edk* b, hipStream_t st);
// ed25519 in-batch key grouping over n items' pub32 (device AoS): table
// (tslots = power of two >= 2n words), rep / uid / slot (n words each),
// count (1 word); the first capU distinct keys' bytes go to kpub32 (32 B each).
hipError_t gvk_ed_group(uint32_t n, const uint8_t* pub32, uint32_t* table, uint32_t tslots, uint32_t* rep,
                        uint32_t* uid, uint32_t* count, uint32_t capU, uint8_t* kpub32, uint32_t* slot,
                        hipStream_t st);
hipError_t gvk_ed_pack_bits(uint32_t n, const uint8_t* out8, uint64_t* bits, hipStream_t st);

hipError_t gvk_gen_gtable(uint32_t* gtab, hipStream_t st);
// the keyed ladder's G tables (GV_KEY2_TABLES x 2 x GV_GTAB_N x 16 words); base_scratch: 48 words
hipError_t gvk_gen_gtable4(uint32_t* gtab4, uint32_t* base_scratch, hipStream_t st);
hipError_t gvk_gen_glat(uint32_t* glat, hipStream_t st);
// the k6 ladder's G tables (GV_K6_GTAB_WORDS words); base_scratch: 112 words
hipError_t gvk_gen_gtable6(uint32_t* gtab6, uint32_t* base_scratch, hipStream_t st);
// The resident arena's k6 tables (GV_KN_ARENA_NG groups of 32 entries) of n
// keys (device pub33) into slots base..base+n-1 (rows of kqt6:
// GV_K6_KEY_WORDS, kqt62: GV_KN_ARENA_NG - 1 per slot, kzq62:
// (GV_KN_ARENA_NG - 1) x 8 rows); scratch as gvk_keys_build.
hipError_t gvk_keys_build6(const uint8_t* pub33, uint32_t n, uint32_t C, uint32_t* in_x, uint32_t* in_pfx,
                           uint32_t* in_r, uint32_t* in_s, uint32_t* in_e, uint32_t* scratch, int with_qe,
                           uint32_t base, uint32_t* kqt6, uint32_t* kzq6, uint32_t kC, uint32_t* kok, uint32_t* kqt62,
                           uint32_t* kzq62, hipStream_t st);
// The resident arena's wide-window tables (ng = GV_KW_NG1 or GV_KW_NG2 groups
// of GV_KW_NT entries), same arguments as gvk_keys_build6 (kqtw:
// GV_KW_KEY_WORDS per slot, kqtw2: ng - 1 rows per slot, kzqw2: (ng - 1) x 8 rows).
hipError_t gvk_keys_build_wide(const uint8_t* pub33, uint32_t n, uint32_t C, uint32_t* in_x, uint32_t* in_pfx,
                           uint32_t* in_r, uint32_t* in_s, uint32_t* in_e, uint32_t* scratch, int with_qe,
                           uint32_t base, uint32_t* kqtw, uint32_t* kzqw, uint32_t kC, uint32_t* kok, uint32_t* kqtw2,
                           uint32_t* kzqw2, int ng, hipStream_t st);
// the full-scalar G tables (GV_GF_WORDS words); base_scratch: 96 words
hipError_t gvk_gen_gtablef(uint32_t* gtabf, uint32_t* base_scratch, hipStream_t st);
// Key-table builds (k_keys_chain + k_keys_fwd + k_keys_back): scratch of
// gvk_keys_scratch_words(n, groups, entries, with_qe) words -- the ratio rows,
// the E rows and (with_qe) the forward entries, all of stride
// gvk_keys_lanes(n, groups) = round_up(groups * n, 256).
uint32_t gvk_keys_lanes(uint32_t n, int ng);
size_t gvk_keys_scratch_words(uint32_t n, int ng, int nt, int with_qe);
// k6 key tables (4 groups of 32 entries) of n keys already unpacked into rows
// in_x / in_pfx (stride C), slots 0..n-1.  kqt: n x GV_K6_KEY_WORDS, kqt2:
// 3 n x GV_K6_KEY_WORDS.
hipError_t gvk_keys_build_rows6(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                                uint32_t* scratch, int with_qe, uint32_t* kqt, uint32_t* kzq, uint32_t kC,
                                uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, hipStream_t st);
// kg key tables (ng groups of 16 entries, ng one of GV_KG_NGS) of n keys
// already unpacked, slots 0..n-1.  kqt: n x GV_KEY_WORDS, kqt2: (ng - 1) n x
// GV_KEY_WORDS, kzq2: (ng - 1) x 8 rows of stride kC.
hipError_t gvk_keys_build_rows_kg(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                                  uint32_t* scratch, int with_qe, uint32_t* kqt, uint32_t* kzq, uint32_t kC,
                                  uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, int ng, hipStream_t st);
hipError_t gvk_verify_lat(const gvk_lat* b, hipStream_t st);
hipError_t gvk_verify_lat16(const gvk_lat* b, hipStream_t st);
hipError_t gvk_verify_lat_sl(const gvk_lat* b, hipStream_t st);
hipError_t gvk_verify_lat16_sl(const gvk_lat* b, hipStream_t st); // keyed, limb-sliced (one signature per block)   // pub33, limb-sliced (one signature per block)
hipError_t gvk_sha256(const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t C,
                      uint32_t* e, hipStream_t st);
hipError_t gvk_verify(const gvk_batch* b, hipStream_t st);
hipError_t gvk_unpack(const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32, uint32_t n, uint32_t C,
                      uint32_t* x, uint32_t* pfx, uint32_t* r, uint32_t* s, uint32_t* e, hipStream_t st);
// In-batch key grouping (gv_kernels.hip k_dedupe*): rep / uid / kslot (n
// words each), table (tslots = power of two >= 2n words), count (1 word); the
// first capU distinct keys' (prefix, x) go to key rows kx (8 rows) / kpfx of
// stride CU.
hipError_t gvk_dedupe(uint32_t n, uint32_t C, const uint32_t* x, const uint32_t* pfx, uint32_t* table, uint32_t tslots,
                      uint32_t* rep, uint32_t* uid, uint32_t* count, uint32_t* kslot, uint32_t capU, uint32_t CU,
                      uint32_t* kx, uint32_t* kpfx, hipStream_t st);
// The k4 key tables (4 groups of 16 entries) of n keys already unpacked into
// rows in_x / in_pfx (stride C), slots 0..n-1 (scratch: gvk_keys_scratch_words).
hipError_t gvk_keys_build_rows(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                               uint32_t* scratch, int with_qe, uint32_t* kqt, uint32_t* kzq, uint32_t kC,
                               uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, hipStream_t st);
// Parse n keys (device pub33) into arena slots base..base+n-1 (k4 tables).
// Scratch: the batch rows in_x, in_pfx (and r, s, e as k_unpack targets) of
// stride C and gvk_keys_scratch_words(n, 4, GV_QTAB_N, with_qe) words.
hipError_t gvk_keys_build(const uint8_t* pub33, uint32_t n, uint32_t C, uint32_t* in_x, uint32_t* in_pfx,
                          uint32_t* in_r, uint32_t* in_s, uint32_t* in_e, uint32_t* scratch, int with_qe,
                          uint32_t base, uint32_t* kqt, uint32_t* kzq, uint32_t kC, uint32_t* kok, uint32_t* kqt2,
                          uint32_t* kzq2, hipStream_t st);
hipError_t gvk_keys_point(uint32_t n, const uint32_t* slots, const uint32_t* kqt, const uint32_t* kzq, uint32_t kC,
                          const uint32_t* kok, uint32_t kcount, uint8_t* out_xy, uint8_t* out_ok, hipStream_t st);
hipError_t gvk_debug(int op, uint32_t n, const uint32_t* in, uint32_t* out, hipStream_t st);
#if GV_STAMP
hipError_t gvk_stamps_read(uint64_t* host, size_t n_u64);   // diagnostic builds (gv_kernels.hip GV_STAMP)
#endif

#ifdef __cplusplus
}
#endif
