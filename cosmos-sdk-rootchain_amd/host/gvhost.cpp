// gvhost.cpp -- host-side mirror of the reference's signature-verification
// ante path and the baseapp batching hooks around it (see gvhost.h for the
// file:line map).  Every secp256k1 leaf of a transaction, a block or a CheckTx
// window is answered from a bounded verdict cache or verified in one
// libgpuverify batch.
//
// Block path (PreVerifyTxs / DeliverBlock): txs are decoded and every
// signer's sign bytes predicted in parallel (sequence = state + earlier txs of
// the same signer in the block), the verdict-cache misses go to the GPU in one
// call with no app lock held, and the decode + per-signer plans are memoised
// so the serial DeliverTx loop only checks each prediction against the state
// and reads the cache.  A wrong prediction is a cache miss, never a different
// verdict: the ante run rebuilds the sign bytes from the actual state.
#include "gvhost.h"

#include <deque>
#include <openssl/evp.h>
#include <openssl/ripemd.h>
#include <openssl/sha.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <time.h>
#include <random>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

using Bytes = std::vector<uint8_t>;
using Addr = std::array<uint8_t, 20>;
using H32 = std::array<uint8_t, 32>;

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
};

// ------------------------------------------------------------------ errors
// sdkerrors codes (types/errors/errors.go)
constexpr uint32_t kErrTxDecode = 2, kErrUnauthorized = 4, kErrInvalidPubKey = 8, kErrUnknownAddress = 9,
                   kErrOutOfGas = 11, kErrMemoTooLarge = 12, kErrTooManySignatures = 14, kErrPanic = 111222;

struct SdkError {
  uint32_t code = 0;
  std::string codespace;
  std::string log;
};

const char* err_desc(uint32_t code) {
  switch (code) {
    case kErrTxDecode: return "tx parse error";
    case kErrUnauthorized: return "unauthorized";
    case kErrInvalidPubKey: return "invalid pubkey";
    case kErrUnknownAddress: return "unknown address";
    case kErrOutOfGas: return "out of gas";
    case kErrMemoTooLarge: return "memo too large";
    case kErrTooManySignatures: return "maximum number of signatures exceeded";
    case kErrPanic: return "panic";
    default: return "internal";
  }
}
// sdkerrors.Wrap(err, msg).Error() == msg + ": " + err.Error()
SdkError wrap(uint32_t code, const std::string& msg) {
  return SdkError{code, code == kErrPanic ? "undefined" : "sdk", msg + ": " + err_desc(code)};
}

// Thrown where the reference panics (amino MustUnmarshal, index out of range,
// nil interface); runTx recovers it into ErrPanic (baseapp/baseapp.go:490-512).
struct Panic : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct OutOfGas {
  std::string descriptor;
};
// go-amino decode error (DefaultTxDecoder wraps it into ErrTxDecode)
struct AminoErr : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------- hashing
// OpenSSL's one-shot SHA256() fetches the digest from the provider store on
// every call (a global lock); the context API hashes with no shared state.
struct Sha256 {
  SHA256_CTX c;
  Sha256() { SHA256_Init(&c); }
  void up(const void* p, size_t n) { SHA256_Update(&c, p, n); }
  void up(const std::string& s) { SHA256_Update(&c, s.data(), s.size()); }
  H32 fin() {
    H32 o;
    SHA256_Final(o.data(), &c);
    return o;
  }
};
H32 sha256(const uint8_t* p, size_t n) {
  Sha256 h;
  h.up(p, n);
  return h.fin();
}

// ------------------------------------------------------------------ bech32
std::string bech32(const std::string& hrp, const uint8_t* data, size_t n);
uint32_t bech32_polymod(const std::vector<uint8_t>& v) {
  static const uint32_t G[5] = {0x3b6a57b2, 0x26508e6d, 0x1ea119fa, 0x3d4233dd, 0x2a1462b3};
  uint32_t chk = 1;
  for (uint8_t x : v) {
    uint32_t b = chk >> 25;
    chk = ((chk & 0x1ffffff) << 5) ^ x;
    for (int i = 0; i < 5; ++i)
      if ((b >> i) & 1) chk ^= G[i];
  }
  return chk;
}
// bech32 of data appended to o (stack buffers, table-driven checksum).
struct Bech32Gen {
  uint32_t t[32];
  Bech32Gen() {
    static const uint32_t G[5] = {0x3b6a57b2, 0x26508e6d, 0x1ea119fa, 0x3d4233dd, 0x2a1462b3};
    for (int b = 0; b < 32; ++b) {
      t[b] = 0;
      for (int k = 0; k < 5; ++k)
        if ((b >> k) & 1) t[b] ^= G[k];
    }
  }
};
const Bech32Gen kBech32Gen;
void bech32_encode_append(std::string& o, const char* hrp, const uint8_t* data, size_t n) {
  static const char* CS = "qpzry9x8gf2tvdw0s3jn54khce6mua7l";
  const size_t hl = strlen(hrp);
  // checksum state after the expanded hrp (hi bits, 0, lo bits)
  uint32_t chk = 1;
  auto step = [&](uint32_t v) { chk = ((chk & 0x1ffffff) << 5) ^ v ^ kBech32Gen.t[chk >> 25]; };
  for (size_t i = 0; i < hl; ++i) step((uint8_t)hrp[i] >> 5);
  step(0);
  for (size_t i = 0; i < hl; ++i) step((uint8_t)hrp[i] & 31);
  char out[16 + 1 + 420 + 6];
  size_t k = 0;
  memcpy(out, hrp, hl);
  k = hl;
  out[k++] = '1';
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < n; ++i) {
    acc = (acc << 8) | data[i];
    bits += 8;
    while (bits >= 5) {
      bits -= 5;
      const uint32_t v = (acc >> bits) & 31;
      step(v);
      out[k++] = CS[v];
    }
  }
  if (bits) {
    const uint32_t v = (acc << (5 - bits)) & 31;
    step(v);
    out[k++] = CS[v];
  }
  for (int i = 0; i < 6; ++i) step(0);
  chk ^= 1;
  for (int i = 0; i < 6; ++i) out[k++] = CS[(chk >> (5 * (5 - i))) & 31];
  o.append(out, k);
}
// "cosmos" addresses repeat (a signer's every tx, a common recipient): a small
// per-thread direct-mapped cache of recent 20-byte encodings.
void bech32_append(std::string& o, const char* hrp, const uint8_t* data, size_t n) {
  if (n != 20 || n > 256 || strcmp(hrp, "cosmos")) {
    if (n > 256) o += bech32(hrp, data, n);
    else bech32_encode_append(o, hrp, data, n);
    return;
  }
  struct Ent {
    uint8_t key[20];
    uint8_t len;
    char s[47];
  };
  static thread_local Ent cache[256];
  uint32_t h;
  memcpy(&h, data + 16, 4);
  Ent& e = cache[(h ^ (h >> 8) ^ data[0]) & 255];
  if (e.len && !memcmp(e.key, data, 20)) { o.append(e.s, e.len); return; }
  const size_t o0 = o.size();
  bech32_encode_append(o, hrp, data, n);
  const size_t len = o.size() - o0;
  if (len <= sizeof e.s) {
    memcpy(e.key, data, 20);
    memcpy(e.s, o.data() + o0, len);
    e.len = (uint8_t)len;
  }
}
std::string bech32(const std::string& hrp, const uint8_t* data, size_t n) {
  static const char* CS = "qpzry9x8gf2tvdw0s3jn54khce6mua7l";
  std::vector<uint8_t> five;
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < n; ++i) {
    acc = (acc << 8) | data[i];
    bits += 8;
    while (bits >= 5) { bits -= 5; five.push_back((acc >> bits) & 31); }
  }
  if (bits) five.push_back((acc << (5 - bits)) & 31);
  std::vector<uint8_t> v;
  for (char c : hrp) v.push_back((uint8_t)c >> 5);
  v.push_back(0);
  for (char c : hrp) v.push_back((uint8_t)c & 31);
  v.insert(v.end(), five.begin(), five.end());
  for (int i = 0; i < 6; ++i) v.push_back(0);
  uint32_t pm = bech32_polymod(v) ^ 1;
  std::string out = hrp + "1";
  for (uint8_t d : five) out += CS[d];
  for (int i = 0; i < 6; ++i) out += CS[(pm >> (5 * (5 - i))) & 31];
  return out;
}
// sdk.AccAddress.String(): "" for an empty address (types/address.go:222-234)
std::string acc_string(const uint8_t* a, size_t n) { return n ? bech32("cosmos", a, n) : std::string(); }
std::string acc_string(Span a) { return acc_string(a.p, a.n); }

// --------------------------------------------------- Go encoding/json strings
// json.Marshal(string): escapes '"', '\\', control chars, HTML <>&, U+2028/9;
// invalid UTF-8 becomes U+FFFD.
void go_json_string(std::string& o, const uint8_t* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  size_t i = 0;
  while (i < n) {
    unsigned char c = s[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
      else if (c == '\n') o += "\\n";
      else if (c == '\r') o += "\\r";
      else if (c == '\t') o += "\\t";
      else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
        o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15];
      } else o += (char)c;
      ++i;
      continue;
    }
    int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    uint32_t cp = 0;
    bool ok = len && i + len <= n;
    if (ok) {
      cp = c & (0x7F >> len);
      for (int k = 1; k < len; ++k) {
        unsigned char cc = s[i + k];
        if ((cc & 0xC0) != 0x80) { ok = false; break; }
        cp = (cp << 6) | (cc & 0x3F);
      }
      if (ok && ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
                 (cp >= 0xD800 && cp <= 0xDFFF)))
        ok = false;
    }
    if (!ok) { o += "\xEF\xBF\xBD"; ++i; continue; }
    if (cp == 0x2028 || cp == 0x2029) o += cp == 0x2028 ? "\\u2028" : "\\u2029";
    else o.append((const char*)s + i, len);
    i += len;
  }
  o += '"';
}
void go_json_string(std::string& o, const std::string& s) { go_json_string(o, (const uint8_t*)s.data(), s.size()); }
std::string go_json_string(const std::string& s) {
  std::string o;
  go_json_string(o, s);
  return o;
}

// ------------------------------------------------------------------- amino
// go-amino v0.15.1 (go.mod:30) binary decoding, restated: uvarint keys
// (field << 3 | typ3), fields in increasing order, repeated (unpacked list)
// fields as consecutive entries, unknown fields only after the known ones,
// registered concrete types behind a 4-byte prefix (optionally preceded by
// 0x00 + 3 disambiguation bytes).

struct Reader {
  const uint8_t* p;
  size_t n, i = 0;
  Reader(Span s) : p(s.p), n(s.n) {}
  bool done() const { return i >= n; }
  uint64_t uvarint() {                        // encoding/binary.Uvarint
    uint64_t x = 0;
    unsigned s = 0;
    for (int k = 0; k < 10; ++k) {
      if (i >= n) throw AminoErr("EOF decoding uvarint");
      const uint8_t b = p[i++];
      if (b < 0x80) {
        if (k == 9 && b > 1) throw AminoErr("EOF decoding uvarint");
        return x | (uint64_t)b << s;
      }
      x |= (uint64_t)(b & 0x7F) << s;
      s += 7;
    }
    throw AminoErr("EOF decoding uvarint");
  }
  void key(uint32_t& f, int& t) {
    const uint64_t v = uvarint();
    t = (int)(v & 7);
    if ((v >> 3) > (1u << 29) - 1) throw AminoErr("invalid field num");
    f = (uint32_t)(v >> 3);
  }
  Span bytes() {
    const uint64_t l = uvarint();
    if (l > n - i) throw AminoErr("insufficient bytes decoding byteslice");
    Span s{p + i, (size_t)l};
    i += (size_t)l;
    return s;
  }
  void skip(int t) {
    switch (t) {
      case 0: uvarint(); break;
      case 1: if (n - i < 8) throw AminoErr("EOF decoding 8 bytes"); i += 8; break;
      case 2: bytes(); break;
      case 5: if (n - i < 4) throw AminoErr("EOF decoding 4 bytes"); i += 4; break;
      default: throw AminoErr("invalid typ3 byte");
    }
  }
};

struct FSpec {
  uint32_t num;
  int typ;
  bool rep;
};
// Walk the fields of one amino struct encoding; fn(field, reader) consumes the value.
template <size_t K, class F>
void for_fields(Span s, const FSpec (&spec)[K], F&& fn) {
  Reader r(s);
  uint32_t last = 0, maxk = 0;
  for (const FSpec& f : spec) maxk = std::max(maxk, f.num);
  while (!r.done()) {
    uint32_t f;
    int t;
    r.key(f, t);
    const FSpec* fs = nullptr;
    for (const FSpec& x : spec)
      if (x.num == f) fs = &x;
    if (!(fs && fs->rep && f == last) && f <= last)
      throw AminoErr("encountered fieldNum: " + std::to_string(f) + ", but we have already seen fnum: " +
                     std::to_string(last));
    last = f;
    if (!fs) {
      if (f < maxk) throw AminoErr("expected field # of struct, got " + std::to_string(f));
      r.skip(t);
      continue;
    }
    if (t != fs->typ) throw AminoErr("expected field type for # " + std::to_string(f));
    fn(f, r);
  }
}

// amino name -> (disambiguation, prefix): SHA256(name), skip zero bytes, 3
// disambiguation bytes, skip zero bytes, 4 prefix bytes.  Reproduces the
// pinned prefixes of crypto/encode_test.go:58-59.
struct Disfix {
  uint8_t d[3], p[4];
};
Disfix disfix(const char* name) {
  const H32 h = sha256((const uint8_t*)name, strlen(name));
  size_t i = 0;
  while (h[i] == 0) ++i;
  Disfix r;
  memcpy(r.d, &h[i], 3);
  i += 3;
  while (h[i] == 0) ++i;
  memcpy(r.p, &h[i], 4);
  return r;
}
const Disfix kSecp = disfix("tendermint/PubKeySecp256k1"), kEd = disfix("tendermint/PubKeyEd25519"),
             kMulti = disfix("tendermint/PubKeyMultisigThreshold"), kStdTx = disfix("cosmos-sdk/StdTx"),
             kMsgSend = disfix("cosmos-sdk/MsgSend"), kMsgMultiSend = disfix("cosmos-sdk/MsgMultiSend");

// Interface value: consumes the disambiguation/prefix bytes; returns the
// registered type among `types` (index) and leaves r at the concrete body.
int interface_type(Span s, Span* body, std::initializer_list<const Disfix*> types) {
  size_t off;
  const uint8_t* pre;
  const uint8_t* dis = nullptr;
  if (s.n >= 8 && s.p[0] == 0x00) { dis = s.p + 1; pre = s.p + 4; off = 8; }
  else if (s.n >= 4) { pre = s.p; off = 4; }
  else throw AminoErr("EOF reading prefix bytes");
  int k = 0;
  for (const Disfix* t : types) {
    if (!memcmp(pre, t->p, 4) && (!dis || !memcmp(dis, t->d, 3))) {
      *body = Span{s.p + off, s.n - off};
      return k;
    }
    ++k;
  }
  throw AminoErr("unrecognized prefix bytes");
}

// ---------------------------------------------------------------- sdk.Int
// Int.Unmarshal (types/int.go:385-405): big.Int.UnmarshalText (Go
// SetString base 0: sign, 0b/0o/0x/0 prefixes, '_' separators) and at most 255
// bits; the sign-bytes JSON then prints the canonical decimal
// (marshalJSON, types/int.go:332-339).  nil (no bytes) prints "0".
std::string int_text_canonical(Span s) {
  if (s.n == 0) return "0";
  if (s.n <= 76 && s.p[0] >= '1' && s.p[0] <= '9') {   // plain decimal < 10^76 < 2^255: already canonical
    bool plain = true;
    for (size_t i = 1; i < s.n && plain; ++i) plain = s.p[i] >= '0' && s.p[i] <= '9';
    if (plain) return std::string((const char*)s.p, s.n);
  }
  const uint8_t* p = s.p;
  size_t i = 0, n = s.n;
  bool neg = false;
  if (p[i] == '+' || p[i] == '-') { neg = p[i] == '-'; ++i; }
  unsigned base = 10;
  char prefix = 0;
  char prev = '.';
  size_t count = 0;
  if (i < n && p[i] == '0') {
    prev = '0';
    count = 1;
    ++i;
    if (i < n) {
      switch (p[i]) {
        case 'b': case 'B': base = 2; prefix = 'b'; break;
        case 'o': case 'O': base = 8; prefix = 'o'; break;
        case 'x': case 'X': base = 16; prefix = 'x'; break;
        default: base = 8; prefix = '0'; break;
      }
      count = 0;
      if (prefix != '0') ++i;
    }
  }
  uint64_t w[5] = {0, 0, 0, 0, 0};                 // magnitude, little-endian 64-bit limbs (320 bits)
  bool inval_sep = false;
  for (; i < n; ++i) {
    const uint8_t ch = p[i];
    if (ch == '_') {
      if (prev != '0') inval_sep = true;
      prev = '_';
      continue;
    }
    unsigned d = 99;
    if (ch >= '0' && ch <= '9') d = ch - '0';
    else if (ch >= 'a' && ch <= 'z') d = ch - 'a' + 10;
    else if (ch >= 'A' && ch <= 'Z') d = ch - 'A' + 10;
    if (d >= base) break;
    prev = '0';
    ++count;
    unsigned __int128 c = d;
    for (auto& x : w) {
      c += (unsigned __int128)x * base;
      x = (uint64_t)c;
      c >>= 64;
    }
    if (c || w[4] >> 32) throw AminoErr("integer out of range");
  }
  if (count == 0 && prefix != '0') throw AminoErr("math/big: cannot unmarshal into a *big.Int");
  if (i != n) throw AminoErr("math/big: cannot unmarshal into a *big.Int");
  if (inval_sep || prev == '_') throw AminoErr("math/big: cannot unmarshal into a *big.Int");
  if (w[4] || (w[3] >> 63)) throw AminoErr("integer out of range");   // BitLen > 255
  std::string dec;
  uint64_t t[4] = {w[0], w[1], w[2], w[3]};
  for (;;) {
    bool zero = !(t[0] | t[1] | t[2] | t[3]);
    if (zero) break;
    unsigned __int128 rem = 0;
    for (int k = 3; k >= 0; --k) {
      unsigned __int128 cur = (rem << 64) | t[k];
      t[k] = (uint64_t)(cur / 10);
      rem = cur % 10;
    }
    dec += (char)('0' + (int)rem);
  }
  if (dec.empty()) return "0";
  if (neg) dec += '-';
  std::reverse(dec.begin(), dec.end());
  return dec;
}

// ------------------------------------------------------------ msgs, StdTx
// sdk.Coin amino (types/types.pb.go:33-36: Denom field 1, Amount field 2);
// JSON {"amount":"N","denom":"d"} with denom omitempty.
void coin_json(std::string& o, Span s) {
  Span denom;
  std::string amount = "0";
  static const FSpec spec[] = {{1, 2, false}, {2, 2, false}};
  for_fields(s, spec, [&](uint32_t f, Reader& r) {
    Span b = r.bytes();
    if (f == 1) denom = b;
    else amount = int_text_canonical(b);
  });
  o += "{\"amount\":\"";
  o += amount;
  o += '"';
  if (denom.n) { o += ",\"denom\":"; go_json_string(o, denom.p, denom.n); }
  o += '}';
}
// sdk.Coins (repeated Coin) as JSON into o: null when absent (amino encodes a
// nil slice as null).  Call add() per element, then done().
struct CoinsJson {
  std::string& o;
  bool any = false;
  explicit CoinsJson(std::string& out) : o(out) {}
  void add(Span c) {
    o += any ? ',' : '[';
    any = true;
    coin_json(o, c);
  }
  void done() { o += any ? "]" : "null"; }
};

void add_signer(std::vector<Span>& signers, Span a) {   // StdTx.GetSigners(): dedupe, first occurrence
  for (const Span& s : signers)
    if (s.n == a.n && !memcmp(s.p, a.p, a.n)) return;
  signers.push_back(a);
}

// x/bank MsgSend (types.pb.go:30-34): from field 1, to field 2, amount field 3;
// GetSignBytes (MustSortJSON of the amino JSON) / GetSigners at x/bank/types/msgs.go:43-50.
// Appends the JSON to o, the signer to signers.
void decode_msg_send(Span body, std::string& o, std::vector<Span>& signers) {
  Span from, to;
  thread_local std::string coins;                 // scratch: capacity reused across txs
  coins.clear();
  CoinsJson cj(coins);
  static const FSpec spec[] = {{1, 2, false}, {2, 2, false}, {3, 2, true}};
  for_fields(body, spec, [&](uint32_t f, Reader& r) {
    Span b = r.bytes();
    if (f == 1) from = b;
    else if (f == 2) to = b;
    else cj.add(b);
  });
  cj.done();
  o += "{\"type\":\"cosmos-sdk/MsgSend\",\"value\":{\"amount\":";
  o += coins;
  if (from.n) { o += ",\"from_address\":\""; bech32_append(o, "cosmos", from.p, from.n); o += '"'; }
  if (to.n) { o += ",\"to_address\":\""; bech32_append(o, "cosmos", to.p, to.n); o += '"'; }
  o += "}}";
  add_signer(signers, from);
}
// x/bank MsgMultiSend: inputs field 1, outputs field 2; Input/Output {address 1, coins 2}
// (types.pb.go:91-94,144-147); GetSigners = input addresses (msgs.go:86-90).
void decode_msg_multisend(Span body, std::string& o, std::vector<Span>& signers) {
  std::string ins, outs;
  bool any_in = false, any_out = false;
  static const FSpec spec[] = {{1, 2, true}, {2, 2, true}};
  for_fields(body, spec, [&](uint32_t f, Reader& r) {
    Span io = r.bytes();
    Span addr;
    std::string coins;
    CoinsJson cj(coins);
    static const FSpec ispec[] = {{1, 2, false}, {2, 2, true}};
    for_fields(io, ispec, [&](uint32_t g, Reader& r2) {
      Span b = r2.bytes();
      if (g == 1) addr = b;
      else cj.add(b);
    });
    cj.done();
    std::string& s = f == 1 ? ins : outs;
    bool& any = f == 1 ? any_in : any_out;
    s += any ? "," : "[";
    any = true;
    s += "{";
    if (addr.n) { s += "\"address\":\""; bech32_append(s, "cosmos", addr.p, addr.n); s += "\","; }
    s += "\"coins\":" + coins + "}";
    if (f == 1) add_signer(signers, addr);
  });
  o += "{\"type\":\"cosmos-sdk/MsgMultiSend\",\"value\":{\"inputs\":";
  o += any_in ? ins + "]" : std::string("null");
  o += ",\"outputs\":";
  o += any_out ? outs + "]" : std::string("null");
  o += "}}";
}

// auth.StdTx (x/auth/types/stdtx.go:147-152): Msgs field 1 (interface list),
// Fee field 2 {Amount 1, Gas 2}, Signatures field 3 {PubKey 1, Signature 2},
// Memo field 4.  Spans point into `raw`: the caller's bytes (alive for the
// call that decoded it) or `own`, a copy kept for the memo table.
struct Tx {
  Bytes own;
  Span raw;
  bool nil_msg = false;
  uint64_t gas = 0;
  size_t memo_len = 0;              // len(GetMemo()) in bytes (ValidateMemoDecorator)
  struct Sig {
    Span pub, sig;
  };
  std::vector<Sig> sigs;
  std::vector<Span> signers;        // StdTx.GetSigners(): msg signers, deduplicated in order
  std::string sb_tail;              // sign bytes after chain_id: ,"fee":..,"memo":..,"msgs":[..],"sequence":"
  Tx() = default;
  void reset() {                    // for reuse (capacities kept)
    own.clear();
    raw = Span{};
    nil_msg = false;
    gas = 0;
    memo_len = 0;
    sigs.clear();
    signers.clear();
    sb_tail.clear();
  }
  Tx(const Tx&) = delete;
  Tx& operator=(const Tx&) = delete;
};

// DefaultTxDecoder (stdtx.go:321-338): cdc.UnmarshalBinaryBare(txBytes, &StdTx{}).
// StdSignBytes (stdtx.go:292-312) pieces are built on the way: the StdSignDoc
// keys are in sorted order and every embedded JSON is canonical, so composing
// them equals MustSortJSON(amino.MarshalJSON(StdSignDoc{...})).
std::shared_ptr<Tx> decode_tx(const uint8_t* p, size_t n, bool copy, std::shared_ptr<Tx> tx = nullptr) {
  if (tx) tx->reset();                              // a recycled Tx (PreVerifyTxs' per-worker pool)
  else tx = std::make_shared<Tx>();
  if (n == 0) throw AminoErr("tx bytes are empty");
  if (copy) {
    tx->own.assign(p, p + n);
    p = tx->own.data();
  }
  tx->raw = Span{p, n};
  if (n < 4 || memcmp(p, kStdTx.p, 4))
    throw AminoErr("UnmarshalBinaryBare expected to read prefix bytes (since it is registered concrete)");
  thread_local std::string msgs, fee;             // scratch: capacity reused across txs
  msgs.clear();
  fee.clear();
  CoinsJson fj(fee);
  bool first_msg = true;
  Span memo;
  static const FSpec spec[] = {{1, 2, true}, {2, 2, false}, {3, 2, true}, {4, 2, false}};
  for_fields(Span{p + 4, n - 4}, spec, [&](uint32_t f, Reader& r) {
    Span b = r.bytes();
    if (f == 1) {
      if (!first_msg) msgs += ',';
      first_msg = false;
      if (b.n == 0) { tx->nil_msg = true; return; }
      Span body;
      const int k = interface_type(b, &body, {&kMsgSend, &kMsgMultiSend});
      if (k == 0) decode_msg_send(body, msgs, tx->signers);
      else decode_msg_multisend(body, msgs, tx->signers);
    } else if (f == 2) {
      static const FSpec fspec[] = {{1, 2, true}, {2, 0, false}};
      for_fields(b, fspec, [&](uint32_t g, Reader& r2) {
        if (g == 1) fj.add(r2.bytes());
        else tx->gas = r2.uvarint();
      });
    } else if (f == 3) {
      Tx::Sig sg;
      static const FSpec sspec[] = {{1, 2, false}, {2, 2, false}};
      for_fields(b, sspec, [&](uint32_t g, Reader& r2) {
        if (g == 1) sg.pub = r2.bytes();
        else sg.sig = r2.bytes();
      });
      tx->sigs.push_back(sg);
    } else {
      memo = b;
    }
  });
  if (tx->nil_msg) tx->signers.clear();
  tx->memo_len = memo.n;
  // StdFee.Bytes() (stdtx.go:47-58): an empty amount is normalised to [] (not null)
  std::string& t = tx->sb_tail;
  t.reserve(64 + fee.size() + msgs.size() + memo.n);
  t = ",\"fee\":{\"amount\":";
  if (fj.any) { t += fee; t += ']'; }
  else t += "[]";
  t += ",\"gas\":\"";
  t += std::to_string(tx->gas);
  t += "\"},\"memo\":";
  go_json_string(t, memo.p, memo.n);
  t += ",\"msgs\":[";
  t += msgs;
  t += "],\"sequence\":\"";
  return tx;
}

// ------------------------------------------------------------- pubkeys
struct PubKey {
  enum Kind { Nil, Secp256k1, Ed25519, Multisig } kind = Nil;
  std::array<uint8_t, 33> secp{};
  std::array<uint8_t, 32> ed{};
  uint64_t k = 0;
  std::vector<PubKey> subs;
};

// crypto.PubKey amino interface (tendermint crypto codec; prefixes pinned by
// crypto/encode_test.go:51-60): secp256k1 [33]byte, ed25519 [32]byte,
// PubKeyMultisigThreshold {K uint field 1, PubKeys []PubKey field 2}.
PubKey decode_pubkey_body(Span s, int depth) {
  if (depth > 16) throw AminoErr("multisig nesting too deep");
  PubKey pk;
  if (s.n == 0) return pk;                          // nil interface (an empty list element)
  Span body;
  const int k = interface_type(s, &body, {&kSecp, &kEd, &kMulti});
  Reader r(body);
  if (k == 0 || k == 1) {
    const size_t want = k == 0 ? 33 : 32;
    Span b = r.bytes();
    if (b.n != want || !r.done()) throw AminoErr("mismatched byte array length");
    if (k == 0) { pk.kind = PubKey::Secp256k1; memcpy(pk.secp.data(), b.p, 33); }
    else { pk.kind = PubKey::Ed25519; memcpy(pk.ed.data(), b.p, 32); }
    return pk;
  }
  pk.kind = PubKey::Multisig;
  static const FSpec spec[] = {{1, 0, false}, {2, 2, true}};
  for_fields(body, spec, [&](uint32_t f, Reader& r2) {
    if (f == 1) pk.k = r2.uvarint();
    else pk.subs.push_back(decode_pubkey_body(r2.bytes(), depth + 1));
  });
  return pk;
}
// amino.MustUnmarshalBinaryBare(bytes, &pk): a decode error panics (stdtx.go:91, account.go:70)
PubKey decode_pubkey(const uint8_t* p, size_t n) {
  try {
    return decode_pubkey_body(Span{p, n}, 0);
  } catch (const AminoErr& e) {
    throw Panic(e.what());
  }
}

void put_uvarint(Bytes& o, uint64_t v) {
  while (v >= 0x80) { o.push_back((uint8_t)(v | 0x80)); v >>= 7; }
  o.push_back((uint8_t)v);
}
// pk.Bytes() = cdc.MustMarshalBinaryBare(pk): the canonical encoding
// (SetPubKey stores it, account.go:75-83; multisig Address hashes it).
void encode_pubkey(Bytes& o, const PubKey& pk) {
  switch (pk.kind) {
    case PubKey::Nil: return;
    case PubKey::Secp256k1:
      o.insert(o.end(), kSecp.p, kSecp.p + 4); o.push_back(33); o.insert(o.end(), pk.secp.begin(), pk.secp.end());
      return;
    case PubKey::Ed25519:
      o.insert(o.end(), kEd.p, kEd.p + 4); o.push_back(32); o.insert(o.end(), pk.ed.begin(), pk.ed.end());
      return;
    case PubKey::Multisig:
      o.insert(o.end(), kMulti.p, kMulti.p + 4);
      if (pk.k) { o.push_back(0x08); put_uvarint(o, pk.k); }
      for (const PubKey& s : pk.subs) {
        Bytes b;
        encode_pubkey(b, s);
        o.push_back(0x12);
        put_uvarint(o, b.size());
        o.insert(o.end(), b.begin(), b.end());
      }
      return;
  }
}
Bytes pubkey_bytes(const PubKey& pk) {
  Bytes b;
  encode_pubkey(b, pk);
  return b;
}

int count_subkeys(const PubKey& pk) {  // types.CountSubKeys (stdtx.go:125-137)
  if (pk.kind != PubKey::Multisig) return 1;
  int c = 0;
  for (auto& s : pk.subs) c += count_subkeys(s);
  return c;
}

Addr pubkey_address(const PubKey& pk) {
  Addr a{};
  if (pk.kind == PubKey::Secp256k1) {
    auto h = sha256(pk.secp.data(), 33);
    RIPEMD160_CTX c;                                  // context API: no provider fetch per call
    RIPEMD160_Init(&c);
    RIPEMD160_Update(&c, h.data(), 32);
    RIPEMD160_Final(a.data(), &c);
  } else if (pk.kind == PubKey::Ed25519) {
    auto h = sha256(pk.ed.data(), 32);
    memcpy(a.data(), h.data(), 20);
  } else if (pk.kind == PubKey::Multisig) {
    Bytes b = pubkey_bytes(pk);
    auto h = sha256(b.data(), b.size());
    memcpy(a.data(), h.data(), 20);
  } else {
    throw Panic("runtime error: invalid memory address or nil pointer dereference");
  }
  return a;
}


// tendermint libs/bits CompactBitArray + crypto/multisig Multisignature
struct CompactBitArray {
  bool present = false;
  uint8_t extra = 0;
  Span elems;
  int size() const {
    if (!present) return 0;
    if (extra == 0) return (int)elems.n * 8;
    return ((int)elems.n - 1) * 8 + extra;
  }
  // GetIndex (libs/bits): indexing Elems past its end panics
  bool get(int i) const {
    if (i < 0 || i >= size()) return false;
    if ((size_t)(i >> 3) >= elems.n) throw Panic("runtime error: index out of range");
    return (elems.p[i >> 3] & (uint8_t)(1u << (7 - (i % 8)))) != 0;
  }
  int true_bits_before(int idx) const {
    int c = 0;
    for (int i = 0; i < idx && i < size(); ++i) c += get(i);
    return c;
  }
};
// Inline storage for the first N elements (a multisig's signatures: no heap
// allocation per decode for up to N sub-signatures).
template <class T, size_t N>
struct SmallVec {
  T inl[N];
  size_t n = 0;
  std::vector<T> more;
  void push_back(const T& v) {
    if (n < N) inl[n] = v;
    else more.push_back(v);
    ++n;
  }
  size_t size() const { return n; }
  const T& operator[](size_t i) const { return i < N ? inl[i] : more[i - N]; }
};
struct Multisignature {
  CompactBitArray bits;
  SmallVec<Span, 16> sigs;
};
Multisignature decode_multisig(Span s) {
  Multisignature m;
  static const FSpec spec[] = {{1, 2, false}, {2, 2, true}};
  for_fields(s, spec, [&](uint32_t f, Reader& r) {
    Span b = r.bytes();
    if (f == 1) {
      m.bits.present = true;
      static const FSpec bspec[] = {{1, 0, false}, {2, 2, false}};
      for_fields(b, bspec, [&](uint32_t g, Reader& r2) {
        if (g == 1) {
          const uint64_t v = r2.uvarint();
          if (v > 255) throw AminoErr("byte overflow");
          m.bits.extra = (uint8_t)v;
        } else {
          m.bits.elems = r2.bytes();
        }
      });
    } else {
      m.sigs.push_back(b);
    }
  });
  return m;
}

// ------------------------------------------------------------- verdict cache
// Bounded verdict cache: key SHA256(kind || pub || sig || SHA256(signBytes))
// (VerifyBytes depends on the message only through its SHA-256 for
// secp256k1, so a cached verdict is exactly the reference's), 8-way buckets
// with CLOCK (second chance) eviction, lock-striped.
class VerdictCache {
 public:
  explicit VerdictCache(size_t entries) { resize(entries); }
  void resize(size_t entries) {
    std::lock_guard<std::mutex> g(resize_mu_);
    size_t nb = 64;
    while (nb * kWays < entries) nb <<= 1;
    std::vector<Bucket> b(nb);
    for (auto& l : locks_) l.lock();
    buckets_.swap(b);
    mask_ = nb - 1;
    count_ = 0;
    for (auto& l : locks_) l.unlock();
  }
  void clear() { resize(capacity()); }
  size_t capacity() const { return buckets_.size() * kWays; }
  size_t size() const { return count_.load(); }
  // 1/0 verdict, -1 miss
  int get(const H32& k) {
    const uint64_t bi = hash(k) & mask_;
    std::lock_guard<std::mutex> g(locks_[bi & (kLocks - 1)]);   // the stripe is a function of the bucket
    Bucket& b = buckets_[bi];
    for (int w = 0; w < kWays; ++w) {
      Entry& e = b.e[w];
      if (e.state && !memcmp(e.key.data(), k.data(), 32)) {
        e.state = (uint8_t)(2 | (e.state & 1) | 4);    // referenced
        return e.state & 1;
      }
    }
    return -1;
  }
  void put(const H32& k, bool v) {
    const uint64_t bi = hash(k) & mask_;
    std::lock_guard<std::mutex> g(locks_[bi & (kLocks - 1)]);   // the stripe is a function of the bucket
    Bucket& b = buckets_[bi];
    for (int w = 0; w < kWays; ++w)
      if (b.e[w].state && !memcmp(b.e[w].key.data(), k.data(), 32)) { b.e[w].state = (uint8_t)(2 | 4 | v); return; }
    for (int w = 0; w < kWays; ++w)
      if (!b.e[w].state) { b.e[w] = Entry{k, (uint8_t)(2 | 4 | v)}; ++count_; return; }
    for (;;) {                                          // CLOCK: clear referenced bits until a victim
      Entry& e = b.e[b.hand];
      b.hand = (uint8_t)((b.hand + 1) % kWays);
      if (e.state & 4) e.state &= (uint8_t)~4;
      else { e = Entry{k, (uint8_t)(2 | 4 | v)}; return; }
    }
  }

 private:
  static constexpr int kWays = 8;
  static constexpr size_t kLocks = 1024;
  struct Entry {
    H32 key;
    uint8_t state;     // bit 1 occupied, bit 0 verdict, bit 2 referenced
  };
  struct Bucket {
    Entry e[kWays] = {};
    uint8_t hand = 0;
  };
  static uint64_t hash(const H32& k) {
    uint64_t h;
    memcpy(&h, k.data(), 8);                          // the key is a SHA-256 output
    return h;
  }
  std::vector<Bucket> buckets_;
  size_t mask_ = 0;
  std::mutex locks_[kLocks];
  std::mutex resize_mu_;
  std::atomic<size_t> count_{0};
};

// ------------------------------------------------------------ verification
// One leaf: VerifyBytes of a secp256k1 (GPU) or ed25519 (CPU) key.
struct Leaf {
  uint8_t kind = 0;                       // 0 secp256k1, 1 ed25519
  std::array<uint8_t, 33> pub{};          // secp: 33 bytes; ed: first 32
  std::array<uint8_t, 64> sig{};
  H32 dig{};                              // SHA256(signBytes), valid when has_dig
  H32 key{};                              // verdict-cache key (computed when first needed)
  bool keyed = false;
  bool has_dig = true;                    // false: secp leaf of a gpu_hash plan, dig computed on first need
  int verdict = -1;
  std::shared_ptr<const std::string> msg; // the sign bytes: ed25519 (SHA-512 runs over them) and gpu_hash secp
};
void ensure_dig(Leaf& L) {
  if (L.has_dig) return;
  Sha256 h;
  h.up(*L.msg);
  L.dig = h.fin();
  L.has_dig = true;
}
void leaf_key(Leaf& L) {
  ensure_dig(L);
  Sha256 h;
  h.up(&L.kind, 1);
  h.up(L.pub.data(), L.kind ? 32 : 33);
  h.up(L.sig.data(), 64);
  h.up(L.dig.data(), 32);
  L.key = h.fin();
  L.keyed = true;
}

// Verification expression for one signer: tendermint VerifyBytes semantics.
struct Node {
  enum Op { Const, LeafRef, And, PanicNode } op = Const;
  bool value = false;
  int leaf = -1;
  std::vector<Node> kids;
};

// Build the node for pk.VerifyBytes(msg, sig) (secp256k1_nocgo.go / ed25519 /
// multisig threshold_pubkey.go) into n (its kids' capacity is reused: a plan
// keeps its node across pooled Memo reuse).  Multisig leaves are AND-ed in bit
// order; since every leaf is a pure function, the AND equals the reference's
// short-circuit.  pre: sig already decoded as a Multisignature (make_plan
// decodes it once for the gas charge and the node).
void build_node(Node& n, const PubKey& pk, const H32& dig, Span sig, std::vector<Leaf>& leaves,
                const Multisignature* pre = nullptr) {
  n.op = Node::Const;
  n.value = false;
  n.leaf = -1;
  n.kids.clear();
  switch (pk.kind) {
    case PubKey::Nil:
      n.op = Node::PanicNode;                         // method call on a nil interface
      return;
    case PubKey::Secp256k1:
    case PubKey::Ed25519: {
      if (sig.n != 64) return;                        // false
      leaves.emplace_back();
      Leaf& L = leaves.back();
      L.kind = pk.kind == PubKey::Ed25519;
      if (L.kind) memcpy(L.pub.data(), pk.ed.data(), 32);
      else L.pub = pk.secp;
      memcpy(L.sig.data(), sig.p, 64);
      L.dig = dig;                                    // key: leaf_key() on first cache use
      n.op = Node::LeafRef;
      n.leaf = (int)leaves.size() - 1;
      return;
    }
    case PubKey::Multisig: {
      Multisignature local;
      const Multisignature* ms = pre;
      if (!ms) {
        try {
          local = decode_multisig(sig);
        } catch (const AminoErr&) {
          return;                                     // UnmarshalBinaryBare error -> false
        }
        ms = &local;
      }
      const int size = ms->bits.size();
      if ((int)pk.subs.size() != size || ms->sigs.size() < pk.k || (int)ms->sigs.size() > size ||
          ms->bits.true_bits_before(size) < (int)pk.k)
        return;                                       // false
      n.op = Node::And;
      n.kids.reserve(ms->sigs.size());
      size_t si = 0;
      for (int i = 0; i < size; ++i) {
        if (!ms->bits.get(i)) continue;
        if (si >= ms->sigs.size()) throw Panic("runtime error: index out of range");
        n.kids.emplace_back();
        build_node(n.kids.back(), pk.subs[i], dig, ms->sigs[si], leaves);
        ++si;
      }
      return;
    }
  }
}

bool eval(const Node& n, const std::vector<Leaf>& leaves) {
  switch (n.op) {
    case Node::Const: return n.value;
    case Node::LeafRef: return leaves[n.leaf].verdict == 1;
    case Node::PanicNode: throw Panic("runtime error: invalid memory address or nil pointer dereference");
    case Node::And:
      for (auto& k : n.kids)
        if (!eval(k, leaves)) return false;
      return true;
  }
  return false;
}

}  // namespace

// ----------------------------------------------------------------- the app
namespace {

// Persistent worker threads: run(parts, fn) calls fn(0..parts-1), part 0 on
// the caller (PreVerifyTxs runs several parallel stages per block; spawning
// threads for each would cost more than the stage).
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i + 1); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }
  void run(int parts, const std::function<void(int)>& fn) {
    parts = std::max(1, std::min(parts, size()));
    if (parts == 1) { fn(0); return; }
    std::lock_guard<std::mutex> one(run_mu_);            // one parallel stage at a time
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      parts_ = parts;
      pending_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* fn;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        if (id >= parts_) continue;
        fn = fn_;
      }
      (*fn)(id);
      std::lock_guard<std::mutex> lk(m_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_, run_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int parts_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

// store/types/gas.go basicGasMeter (limit) / infiniteGasMeter
struct GasMeter {
  bool infinite;
  uint64_t limit;
  uint64_t used = 0;
  void consume(uint64_t amount, const char* desc) {
    used += amount;
    if (!infinite && used > limit) throw OutOfGas{desc};
  }
  bool fits(uint64_t amount) const { return infinite || used + amount <= limit; }
};

// KV-store gas of the ante chain.  ctx.KVStore wraps every store in gaskv
// (types/context.go:211-212), whose Get charges ReadCostFlat + ReadCostPerByte
// x len(value) and Set WriteCostFlat + WriteCostPerByte x len(value)
// (store/gaskv/store.go:36-52; KVGasConfig store/types/gas.go:165-173).
constexpr uint64_t kReadCostFlat = 1000, kReadCostPerByte = 3, kWriteCostFlat = 2000, kWriteCostPerByte = 30;
constexpr uint64_t kTxSizeCostPerByte = 10, kMaxMemoCharacters = 256;   // x/auth/types/params.go:16,18
void kv_read(GasMeter& gm, size_t value_len) {
  gm.consume(kReadCostFlat, "ReadFlat");
  gm.consume(kReadCostPerByte * value_len, "ReadPerByte");
}
void kv_write(GasMeter& gm, size_t value_len) {
  gm.consume(kWriteCostFlat, "WriteFlat");
  gm.consume(kWriteCostPerByte * value_len, "WritePerByte");
}
size_t uvarint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}
// The value AccountKeeper.SetAccount stores (x/auth/keeper/account.go:51-61):
// std.Codec.MarshalAccount (std/codec.go:41-48) = proto std.Account{base_account
// = 1: BaseAccount{address = 1, pub_key = 2, account_number = 3, sequence = 4}}
// (std/codec.proto:21-32, x/auth/types/types.proto:11-19); proto3 leaves out
// empty and zero fields.  pub_key holds pubKey.Bytes() (amino, account.go:75-83).
size_t account_value_len(size_t pub_len, uint64_t num, uint64_t seq) {
  size_t inner = 2 + 20;
  if (pub_len) inner += 1 + uvarint_len(pub_len) + pub_len;
  if (num) inner += 1 + uvarint_len(num);
  if (seq) inner += 1 + uvarint_len(seq);
  return 1 + uvarint_len(inner) + inner;
}
// AccountKeeper.GetParams (x/auth/keeper/keeper.go GetParams -> params
// Subspace.GetParamSet, x/params/types/subspace.go:100-109,218-222): one
// gas-metered Get per ParamSetPair in x/auth/types/params.go:55-62 order; the
// values are amino JSON (codec/hybrid_codec.go:51-53), uint64 as a quoted
// decimal string.
size_t amino_json_u64_len(uint64_t v) { return std::to_string(v).size() + 2; }

// 64-bit hash of a byte string for in-process tables (entries are always
// confirmed by a full comparison, so collisions cost time, never results).
uint64_t fast_hash(const uint8_t* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = (h ^ (w * 0x87C37B91114253D5ull)) * 0x4CF5AD432745937Full;
    h ^= h >> 31;
  }
  uint64_t w = 0;
  memcpy(&w, p + i, n - i);
  h = (h ^ (w * 0x87C37B91114253D5ull)) * 0x4CF5AD432745937Full;
  return h ^ (h >> 29);
}

// GVH_PROFILE laps: wall time, or (GVH_PROFILE=cpu) the calling thread's CPU
// time -- with one host thread every stage runs on the caller, so the CPU
// clock gives the front's cost without the scheduler's noise
// (tools/front_cost.py).
double prof_ms() {
  static const bool cpu = [] {
    const char* e = getenv("GVH_PROFILE");
    return e && !strcmp(e, "cpu");
  }();
  timespec ts;
  clock_gettime(cpu ? CLOCK_THREAD_CPUTIME_ID : CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

// Open-addressing map from a K-byte public key to a key-arena slot (the
// account key caches below): one flat array probed linearly, so a lookup costs
// about one cache miss -- the node-based unordered_map it replaces took ~20 %
// of a single-threaded C4 block's host front in its bucket walks
// (tools/front_cost, profiles/r06/front_cost).  The hash mixes 16 key bytes
// with a per-process random seed: keys are attacker-chosen (a mempool tx
// names any pubkey), so probe sequences must not be predictable.  Load factor
// <= 1/2; erase shifts the run back (no tombstones).  Not thread-safe: the
// callers' key_mu / gpu_mu rules apply as before (concurrent finds only).
template <size_t K>
class FlatSlotMap {
 public:
  FlatSlotMap() { grow(1024); }
  const uint32_t* find(const uint8_t* key) const {
    for (size_t i = hash(key) & mask_;; i = (i + 1) & mask_) {
      const Ent& e = t_[i];
      if (!e.full) return nullptr;
      if (!memcmp(e.key, key, K)) return &e.val;
    }
  }
  // (slot of the key, inserted?) -- an existing key keeps its value
  std::pair<uint32_t*, bool> emplace(const uint8_t* key, uint32_t val) {
    if (2 * (n_ + 1) > t_.size()) grow(2 * t_.size());
    for (size_t i = hash(key) & mask_;; i = (i + 1) & mask_) {
      Ent& e = t_[i];
      if (!e.full) {
        e.full = 1;
        memcpy(e.key, key, K);
        e.val = val;
        ++n_;
        return {&e.val, true};
      }
      if (!memcmp(e.key, key, K)) return {&e.val, false};
    }
  }
  void set(const uint8_t* key, uint32_t val) { *emplace(key, val).first = val; }
  void erase(const uint8_t* key) {
    size_t i = hash(key) & mask_;
    for (;; i = (i + 1) & mask_) {
      if (!t_[i].full) return;
      if (!memcmp(t_[i].key, key, K)) break;
    }
    // backward-shift deletion: move later members of the run into the hole
    // when their home slot does not lie cyclically in (hole, j]
    for (size_t j = (i + 1) & mask_;; j = (j + 1) & mask_) {
      if (!t_[j].full) break;
      const size_t home = hash(t_[j].key) & mask_;
      const bool stays = i <= j ? (home > i && home <= j) : (home > i || home <= j);
      if (stays) continue;
      t_[i] = t_[j];
      i = j;
    }
    t_[i].full = 0;
    --n_;
  }
  void clear() {
    for (Ent& e : t_) e.full = 0;
    n_ = 0;
  }
  size_t size() const { return n_; }

 private:
  struct Ent {
    uint32_t val;
    uint8_t full;
    uint8_t key[K];
  };
  uint64_t hash(const uint8_t* key) const {
    constexpr size_t o = K == 33 ? 1 : 0;                 // skip a compressed key's prefix byte
    uint64_t w0, w1;
    memcpy(&w0, key + o, 8);
    memcpy(&w1, key + o + 8, 8);
    uint64_t h = (w0 ^ seed_) * 0x87C37B91114253D5ull;
    h = (h ^ (h >> 31) ^ w1) * 0x4CF5AD432745937Full;
    return h ^ (h >> 29);
  }
  void grow(size_t cap) {
    std::vector<Ent> old;
    old.swap(t_);
    t_.assign(cap, Ent{});
    mask_ = cap - 1;
    n_ = 0;
    for (const Ent& e : old)
      if (e.full) emplace(e.key, e.val);
  }
  std::vector<Ent> t_;
  size_t n_ = 0, mask_ = 0;
  const uint64_t seed_ = ((uint64_t)std::random_device{}() << 32) ^ std::random_device{}();
};

// A decoded amino pubkey with its canonical bytes (pk.Bytes()), address and
// CountSubKeys -- pure functions of the amino bytes, shared by every tx and
// account that carries the same key.
struct PubInfo {
  Bytes raw;                    // the amino bytes it was decoded from
  PubKey pk;
  Bytes canon;
  Addr addr{};
  int subkeys = 1;
};
class PubCache {
 public:
  // throws Panic if the bytes do not decode (MustUnmarshalBinaryBare)
  std::shared_ptr<const PubInfo> get(const uint8_t* p, size_t n) {
    const uint64_t h = fast_hash(p, n);
    Shard& s = shards_[h & (kShards - 1)];
    {
      std::lock_guard<std::mutex> g(s.mu);
      auto it = s.map.find(h);
      if (it != s.map.end())
        for (auto& e : it->second)
          if (e->raw.size() == n && !memcmp(e->raw.data(), p, n)) return e;
    }
    auto info = std::make_shared<PubInfo>();
    info->raw.assign(p, p + n);
    info->pk = decode_pubkey(p, n);
    info->canon = pubkey_bytes(info->pk);
    if (info->pk.kind != PubKey::Nil) info->addr = pubkey_address(info->pk);
    info->subkeys = count_subkeys(info->pk);
    std::lock_guard<std::mutex> g(s.mu);
    if (s.count >= kPerShard) { s.map.clear(); s.count = 0; }
    s.map[h].push_back(info);
    ++s.count;
    return info;
  }

 private:
  static constexpr size_t kShards = 64, kPerShard = 8192;
  struct Shard {
    std::mutex mu;
    std::unordered_map<uint64_t, std::vector<std::shared_ptr<const PubInfo>>> map;
    size_t count = 0;
  };
  Shard shards_[kShards];
};

struct Account {
  uint64_t number = 0, sequence = 0;
  Bytes pub;                                  // amino (canonical), empty = not set
  std::shared_ptr<const PubInfo> info;        // GetPubKey() of pub (decoded once)
  uint64_t bump_epoch = 0, bump = 0;          // PreVerifyTxs' sequence prediction (earlier txs this call)
  // Prediction carried across a pipelined replay (deliver_blocks): block E+1
  // is pre-verified before block E is delivered, so its prediction adds
  // block E's effects -- own = txs of block own_epoch signed by this account,
  // own_info = the key its SetPubKey would store -- to the state.
  uint64_t own_epoch = 0, own = 0;
  std::shared_ptr<const PubInfo> own_info, pred_info;   // pred_info: predicted key for bump_epoch
};
// AccountKeeper store: 20-byte address -> Account.  Open addressing (linear
// probing) over an index into a deque, so an Account never moves (PreVerifyTxs
// and the ante loop keep Account pointers) and a lookup is one hash + one or
// two cache lines instead of a node-based map's bucket chain.
class AccountTable {
 public:
  Account* find(const uint8_t* a) {
    if (!n_) return nullptr;
    for (size_t i = fast_hash(a, 20) & mask_;; i = (i + 1) & mask_) {
      const uint32_t s = slots_[i];
      if (!s) return nullptr;
      Entry& e = store_[s - 1];
      if (!memcmp(e.addr.data(), a, 20)) return &e.acc;
    }
  }
  Account& get_or_insert(const Addr& a) {
    if (Account* p = find(a.data())) return *p;
    if ((n_ + 1) * 2 > slots_.size()) grow();
    store_.push_back(Entry{a, Account{}});
    ++n_;
    place(a.data(), (uint32_t)n_);
    return store_.back().acc;
  }

 private:
  struct Entry {
    Addr addr;
    Account acc;
  };
  void place(const uint8_t* a, uint32_t idx) {
    size_t i = fast_hash(a, 20) & mask_;
    while (slots_[i]) i = (i + 1) & mask_;
    slots_[i] = idx;
  }
  void grow() {
    const size_t cap = std::max<size_t>(1024, slots_.size() * 2);
    slots_.assign(cap, 0);
    mask_ = cap - 1;
    for (size_t k = 0; k < n_; ++k) place(store_[k].addr.data(), (uint32_t)(k + 1));
  }
  std::deque<Entry> store_;
  std::vector<uint32_t> slots_;
  size_t mask_ = 0, n_ = 0;
};

// One signer's prepared verification: the sign bytes were built for
// (accnum, seq) with the account pubkey `pub` (its canonical bytes), the gas
// consumer's charge for that key and these signature bytes, and the leaves
// (verdicts filled by PreVerifyTxs' GPU batch).
struct SignerPlan {
  bool ok = false;                  // plan built (else: recompute in ante)
  uint64_t accnum = 0, seq = 0;
  std::shared_ptr<const PubInfo> pub;
  uint64_t gas = 0;
  uint8_t gas_status = 0;           // 0 charged without error, 1 top-level error, 2 panic
  bool resolved = false;            // every leaf has its verdict
  int16_t owner = 0;                // pool worker that built it (release_memos)
  Node node;
  std::vector<Leaf> leaves;
};
// PreVerifyTxs' work on one tx, reused by its ante run.
struct Memo {
  std::shared_ptr<const Tx> tx;
  std::string decode_err;                            // non-empty: the tx did not decode
  std::vector<std::shared_ptr<const PubInfo>> tx_pk; // GetPubKeys(): per StdSignature (null: none)
  int pk_panic = -1;                                 // first tx-supplied key that does not decode
  std::string pk_panic_msg;
  std::vector<SignerPlan> plans;
  std::vector<Account*> sacc;                        // PreVerifyTxs: each signer's account (null: none)
  int16_t owner = 0;                                 // pool worker that decoded it (release_memos)
  void reset() {                                     // for reuse: every field as new, capacities kept
    tx.reset();
    decode_err.clear();
    tx_pk.clear();
    pk_panic = -1;
    pk_panic_msg.clear();
    for (SignerPlan& p : plans) {
      p.ok = false;
      p.accnum = p.seq = 0;
      p.pub.reset();
      p.gas = 0;
      p.gas_status = 0;
      p.resolved = false;
      p.owner = 0;
      p.node.op = Node::Const;                       // the kids' capacity is kept (build_node)
      p.node.kids.clear();
      p.leaves.clear();
    }
    sacc.clear();
    owner = 0;
  }
};

// Memo table (CheckTx window and separate PreVerifyTxs / ante calls): tx
// bytes -> Memo with full-byte comparison, two generations.
class MemoTable {
 public:
  std::shared_ptr<Memo> find(const uint8_t* p, size_t n) {
    const uint64_t h = fast_hash(p, n);
    std::lock_guard<std::mutex> g(mu_);
    for (auto* m : {&cur_, &old_}) {
      auto it = m->find(h);
      if (it != m->end())
        for (auto e = it->second.rbegin(); e != it->second.rend(); ++e)     // newest first
          if ((*e)->tx->raw.n == n && !memcmp((*e)->tx->raw.p, p, n)) return *e;
    }
    return nullptr;
  }
  void put(std::shared_ptr<Memo> m) {
    if (!m->tx) return;
    const uint64_t h = fast_hash(m->tx->raw.p, m->tx->raw.n);
    std::lock_guard<std::mutex> g(mu_);
    if (count_ >= limit_) {
      old_.swap(cur_);
      cur_.clear();
      count_ = 0;
    }
    auto& v = cur_[h];
    for (auto& e : v)
      if (e->tx->raw.n == m->tx->raw.n && !memcmp(e->tx->raw.p, m->tx->raw.p, m->tx->raw.n)) { e = std::move(m); return; }
    v.push_back(std::move(m));
    ++count_;
  }
  void clear() {
    std::lock_guard<std::mutex> g(mu_);
    cur_.clear();
    old_.clear();
    count_ = 0;
  }

 private:
  std::mutex mu_;
  std::unordered_map<uint64_t, std::vector<std::shared_ptr<Memo>>> cur_, old_;
  size_t count_ = 0, limit_ = 1 << 16;
};

struct Window {
  std::mutex m;
  std::condition_variable cv;
  size_t max_txs = 64;
  int64_t max_wait_us = 200;
  // Adaptive: a call waits for company only when calls are concurrent
  // (another one in flight, or the last window held more than one).
  std::atomic<int> inflight{0};
  std::atomic<size_t> last_size{0};
  struct Batch {
    std::vector<std::pair<const uint8_t*, size_t>> items;
    std::chrono::steady_clock::time_point deadline;
    bool flushing = false, done = false;
  };
  std::shared_ptr<Batch> open;
};

// simSecp256k1Pubkey (x/auth/ante/sigverify.go:27-31), amino
const Bytes kSimPub = {0xEB, 0x5A, 0xE9, 0x87, 0x21, 0x03, 0x5A, 0xD6, 0x81, 0x0A, 0x47, 0xF0, 0x73,
                       0x55, 0x3F, 0xF3, 0x0D, 0x2F, 0xCC, 0x7E, 0x0D, 0x3B, 0x1C, 0x0B, 0x74, 0xB6,
                       0x1A, 0x1A, 0xAA, 0x25, 0x82, 0x34, 0x40, 0x37, 0x15, 0x1E, 0x14, 0x3A};

}  // namespace

struct gvh_app {
  gv_ctx* gpu = nullptr;
  uint64_t sig_limit = 7, cost_secp = 1000, cost_ed = 590;
  bool kv_gas = true;                          // charge the ante chain's KV-store and tx-size gas (gvh_set_gas_model)
  std::string chain_id = "", chain_json = "\"\"";
  int64_t height = 1;
  bool recheck = false;
  uint64_t gas_limit = 0;
  AccountTable accounts;                       // AccountKeeper (20-byte addresses)
  std::mutex mu;                               // accounts + context
  VerdictCache cache{size_t(1) << 20};
  MemoTable memo;
  PubCache pubs;
  Window window;
  std::mutex gpu_mu;                           // one GPU batch at a time per app
  // account key cache: pub33 -> key-arena slot of the GPU
  // context (gv_keys_load); guarded by gpu_mu.  keyed = 0: pub33 batches.
  FlatSlotMap<33> key_slots;
  // ed25519 keys (IBC validator sets, multisig ed25519 sub-keys): pub32 ->
  // slot of the context's ed25519 key arena (gv_ed_keys_load); gpu_mu
  FlatSlotMap<32> ed_slots;
  uint64_t ed_key_gen = 0;
  uint64_t key_gen = 0;                        // gv_keys_generation the map belongs to
  bool keyed = true;
  // PreVerifyTxs of a delivered block (keep == false) with an empty verdict
  // cache: secp256k1 sign bytes hashed by the GPU batch (gv_verify_msgs*)
  // rather than on the host (the digest would serve no cache key).  Off by
  // default: measured slower (DESIGN.md §6.5 -- OpenSSL's SHA-256 costs less
  // per tx than building the sign-bytes string and shipping it to the GPU)
  bool gpu_hash = getenv("GVH_GPU_HASH") ? atoi(getenv("GVH_GPU_HASH")) != 0 : false;
  size_t key_cap = GV_KEY_CAP;                 // arena reset past this many keys (5.4 KB of HBM each)
  size_t key_load_min = GV_KEY_LOAD_MIN;       // smaller batches never load keys (k_keys_build's ~ms latency):
                                               // keyed only when all their keys are resident
  int threads = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
  std::unique_ptr<Pool> pool{new Pool(threads - 1)};
  std::mutex pool_mu;                          // guards replacing the pool (gvh_set_threads)
  // Recycled Memo / Tx objects per pool worker (PreVerifyTxs allocates ~10
  // objects per tx; reusing them keeps their vectors' capacity and takes
  // malloc/free off the block path).  Index: worker id & 63.
  struct ObjPool {
    std::mutex mu;
    std::vector<std::shared_ptr<Memo>> memos;
    std::vector<std::shared_ptr<Tx>> txs;
  };
  std::array<ObjPool, 64> objs;
  uint64_t bump_epoch = 0;
  uint64_t carry_epoch = 0;                    // a pre-verified block not yet delivered (deliver_blocks), 0: none
  // key_slots readers (slot lookups on the pool, before the GPU lock) share
  // key_mu; verify_secp's updates take it exclusively (under gpu_mu)
  std::shared_mutex key_mu;
  // pinned pack buffers (gv_host_alloc): the GPU batch reads them in place, no staging copy
  struct PinBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
  };
  std::mutex pin_mu;
  std::vector<PinBuf> pin_free;
  ~gvh_app() {
    for (PinBuf& b : pin_free) {
      if (b.pinned) gv_host_free(gpu, b.p);
      else free(b.p);
    }
  }
  std::atomic<uint64_t> st_gpu_calls{0}, st_gpu_leaves{0}, st_hits{0}, st_misses{0}, st_memo{0}, st_windows{0},
      st_window_txs{0}, st_pre_ns{0}, st_gpu_ns{0}, st_loop_ns{0};
  // the last delivered block's memos, released (back to the worker pools)
  // while the next block's GPU batch runs instead of on the block's own
  // critical path (deliver_block); declared last: dropped first
  std::mutex deferred_mu;
  std::vector<std::shared_ptr<Memo>> deferred;
  bool defer_release = getenv("GVH_DEFER_RELEASE") ? atoi(getenv("GVH_DEFER_RELEASE")) != 0 : true;
  // gvh_deliver_blocks queues block b+1's secp256k1 batch with gv_submit_* and
  // waits for it after block b's loop (no helper thread); 0: a helper thread
  // runs the synchronous call (also the path of batches with ed25519 leaves)
  bool async_blocks = getenv("GVH_ASYNC_BLOCKS") ? atoi(getenv("GVH_ASYNC_BLOCKS")) != 0 : true;
};

namespace {

constexpr size_t kObjPoolCap = size_t(1) << 15;   // per worker
std::shared_ptr<Memo> memo_get(gvh_app* app, int w) {
  auto& p = app->objs[w & 63];
  std::lock_guard<std::mutex> g(p.mu);
  if (p.memos.empty()) return std::make_shared<Memo>();
  auto m = std::move(p.memos.back());
  p.memos.pop_back();
  return m;
}
std::shared_ptr<Tx> tx_get(gvh_app* app, int w) {
  auto& p = app->objs[w & 63];
  std::lock_guard<std::mutex> g(p.mu);
  if (p.txs.empty()) return nullptr;
  auto t = std::move(p.txs.back());
  p.txs.pop_back();
  return t;
}
// m: a memo nobody else holds; back to worker w's pool (its Tx too when unshared)
void memo_put(gvh_app* app, int w, std::shared_ptr<Memo>&& m) {
  std::shared_ptr<Tx> t;
  if (m->tx && m->tx.use_count() == 1) t = std::const_pointer_cast<Tx>(std::move(m->tx));
  m->reset();
  auto& p = app->objs[w & 63];
  std::lock_guard<std::mutex> g(p.mu);
  if (p.memos.size() < kObjPoolCap) p.memos.push_back(std::move(m));
  if (t && p.txs.size() < kObjPoolCap) p.txs.push_back(std::move(t));
  m.reset();
}

// Run fn(i) for i in [0, n) on the app's pool (dynamic chunks).  Nested calls
// (from inside a pool task) run inline.
thread_local bool t_in_pool = false;
template <class F>
void parallel_for(gvh_app* app, size_t n, F fn) {
  const size_t chunk = 16;
  if (app->threads <= 1 || n <= chunk || t_in_pool) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::function<void(int)> work = [&](int) {
    const bool was = t_in_pool;
    t_in_pool = true;
    for (size_t lo; (lo = next.fetch_add(chunk)) < n;)
      for (size_t i = lo; i < std::min(n, lo + chunk); ++i) fn(i);
    t_in_pool = was;
  };
  std::lock_guard<std::mutex> g(app->pool_mu);
  app->pool->run((int)std::min<size_t>(app->threads, (n + chunk - 1) / chunk), work);
}
// parallel_for with the worker's index w in [0, app->threads) as fn(i, w).
template <class F>
void parallel_for_w(gvh_app* app, size_t n, F fn) {
  const size_t chunk = 16;
  if (app->threads <= 1 || n <= chunk || t_in_pool) {
    for (size_t i = 0; i < n; ++i) fn(i, 0);
    return;
  }
  std::atomic<size_t> next{0};
  std::function<void(int)> work = [&](int w) {
    const bool was = t_in_pool;
    t_in_pool = true;
    for (size_t lo; (lo = next.fetch_add(chunk)) < n;)
      for (size_t i = lo; i < std::min(n, lo + chunk); ++i) fn(i, w);
    t_in_pool = was;
  };
  std::lock_guard<std::mutex> g(app->pool_mu);
  app->pool->run((int)std::min<size_t>(app->threads, (n + chunk - 1) / chunk), work);
}
// Run fn(w, nw) once on every pool worker (w = the worker's thread index,
// stable across calls: part 0 is the caller).
template <class F>
void parallel_workers(gvh_app* app, F fn) {
  if (app->threads <= 1 || t_in_pool) {
    fn(0, 1);
    return;
  }
  const int nw = app->threads;
  std::function<void(int)> work = [&](int w) {
    const bool was = t_in_pool;
    t_in_pool = true;
    fn(w, nw);
    t_in_pool = was;
  };
  std::lock_guard<std::mutex> g(app->pool_mu);
  app->pool->run(nw, work);
}
// Run fn(part) for part in [0, parts) on the pool (static partition).
template <class F>
void parallel_parts(gvh_app* app, int parts, F fn) {
  if (parts <= 1 || t_in_pool) {
    for (int p = 0; p < parts; ++p) fn(p);
    return;
  }
  std::atomic<int> next{0};
  std::function<void(int)> work = [&](int) {
    const bool was = t_in_pool;
    t_in_pool = true;
    for (int p; (p = next.fetch_add(1)) < parts;) fn(p);
    t_in_pool = was;
  };
  std::lock_guard<std::mutex> g(app->pool_mu);
  app->pool->run(std::min(parts, app->threads), work);
}

// DefaultSigVerificationGasConsumer (sigverify.go:299-322) incl. the multisig
// recursion (ConsumeMultisignatureVerificationGas :325-338, whose nested errors
// are ignored).  Returns false + err for the top level only.
bool consume_sig_gas(GasMeter& gm, Span sig, const PubKey& pk, const gvh_app* app, SdkError* err,
                     const Multisignature* pre = nullptr) {
  switch (pk.kind) {
    case PubKey::Ed25519:
      gm.consume(app->cost_ed, "ante verify: ed25519");
      if (err) *err = wrap(kErrInvalidPubKey, "ED25519 public keys are unsupported");
      return false;
    case PubKey::Secp256k1:
      gm.consume(app->cost_secp, "ante verify: secp256k1");
      return true;
    case PubKey::Multisig: {
      Multisignature local;
      const Multisignature* ms = pre;
      if (!ms) {
        try {
          local = decode_multisig(sig);              // MustUnmarshalBinaryBare: panics on error
        } catch (const AminoErr& e) {
          throw Panic(e.what());
        }
        ms = &local;
      }
      const int size = ms->bits.size();
      size_t si = 0;
      for (int i = 0; i < size; ++i) {
        if (!ms->bits.get(i)) continue;
        if (si >= ms->sigs.size() || i >= (int)pk.subs.size()) throw Panic("runtime error: index out of range");
        consume_sig_gas(gm, ms->sigs[si], pk.subs[i], app, nullptr);
        ++si;
      }
      return true;
    }
    case PubKey::Nil:
      if (err) *err = wrap(kErrInvalidPubKey, "unrecognized public key type: <nil>");
      return false;
  }
  return true;
}

void copy_result(gvh_result* out, const SdkError* e, uint64_t gas, uint32_t gpu_leaves, uint32_t hits,
                 uint64_t wanted) {
  out->code = 0;
  out->codespace[0] = 0;
  out->log[0] = 0;
  if (e) {
    out->code = e->code;
    snprintf(out->codespace, sizeof out->codespace, "%s", e->codespace.c_str());
    snprintf(out->log, sizeof out->log, "%s", e->log.c_str());
  }
  out->gas_used = gas;
  out->gpu_leaves = gpu_leaves;
  out->cache_hits = hits;
  out->gas_wanted = wanted;
}

Account* find_account(gvh_app* app, Span a) {
  if (a.n != 20) return nullptr;                    // accounts have 20-byte addresses
  return app->accounts.find(a.p);
}

std::shared_ptr<const PubInfo> account_info(gvh_app* app, Account& acc) {
  if (acc.pub.empty()) return nullptr;
  if (!acc.info) acc.info = app->pubs.get(acc.pub.data(), acc.pub.size());
  return acc.info;
}

// Sign-bytes digest of tx for (accnum, seq) on chain_json.
H32 sign_digest(const Tx& tx, const std::string& chain_json, uint64_t accnum, uint64_t seq) {
  char a[24], s[24];
  const int na = snprintf(a, sizeof a, "%llu", (unsigned long long)accnum);
  const int ns = snprintf(s, sizeof s, "%llu", (unsigned long long)seq);
  Sha256 h;
  h.up("{\"account_number\":\"", 19);
  h.up(a, na);
  h.up("\",\"chain_id\":", 13);
  h.up(chain_json);
  h.up(tx.sb_tail);
  h.up(s, ns);
  h.up("\"}", 2);
  return h.fin();
}
std::string sign_bytes(const Tx& tx, const std::string& chain_json, uint64_t accnum, uint64_t seq) {
  return "{\"account_number\":\"" + std::to_string(accnum) + "\",\"chain_id\":" + chain_json + tx.sb_tail +
         std::to_string(seq) + "\"}";
}

// Build a signer's plan: gas charge, sign bytes digest, leaves + keys.
// ed25519 leaves keep the sign bytes themselves (the GPU's SHA-512 runs over
// them); every leaf is then decided by the cache or a GPU batch in resolve().
// gpu_hash: the secp256k1 leaves keep the sign bytes too and no digest (the
// GPU batch hashes them, gv_verify_msgs*); ensure_dig() computes it if the
// leaf meets the cache after all.
void make_plan(SignerPlan& p, gvh_app* app, const Tx& tx, size_t signer, std::shared_ptr<const PubInfo> pub,
               uint64_t accnum, uint64_t seq, const std::string& chain_json, bool gpu_hash = false) {
  p.accnum = accnum;
  p.seq = seq;
  p.pub = std::move(pub);
  p.leaves.clear();
  p.resolved = false;
  // a multisig's signature decoded once, for the gas charge and the node (a
  // decode error: both decode again and fail as the reference does)
  Multisignature pre;
  bool have_pre = false;
  if (p.pub->pk.kind == PubKey::Multisig) {
    try {
      pre = decode_multisig(tx.sigs[signer].sig);
      have_pre = true;
    } catch (const AminoErr&) {
    }
  }
  try {
    GasMeter g{true, 0};
    p.gas_status =
        consume_sig_gas(g, tx.sigs[signer].sig, p.pub->pk, app, nullptr, have_pre ? &pre : nullptr) ? 0 : 1;
    p.gas = g.used;
  } catch (const Panic&) {
    p.gas_status = 2;
  }
  const H32 dig = gpu_hash ? H32{} : sign_digest(tx, chain_json, accnum, seq);
  p.leaves.reserve((size_t)std::max(1, p.pub->subkeys));
  build_node(p.node, p.pub->pk, dig, tx.sigs[signer].sig, p.leaves, have_pre ? &pre : nullptr);
  bool need_msg = false;
  for (const Leaf& L : p.leaves) need_msg = need_msg || L.kind || gpu_hash;
  if (need_msg) {
    auto sb = std::make_shared<const std::string>(sign_bytes(tx, chain_json, accnum, seq));
    for (Leaf& L : p.leaves) {
      if (L.kind || gpu_hash) L.msg = sb;
      if (gpu_hash) L.has_dig = false;            // either kind: the cache key hashes the digest
    }
  }
  p.ok = true;
}

// Verdict-cache lookup / insert of one leaf.  The key (three SHA-256 blocks)
// is computed only when the cache is used: a lookup in an empty cache is a
// miss without hashing (block replay with no CheckTx history).
int cache_lookup(gvh_app* app, Leaf& L) {
  if (app->cache.size() == 0) return -1;
  if (!L.keyed) leaf_key(L);
  return app->cache.get(L.key);
}
void cache_insert(gvh_app* app, Leaf& L, bool v) {
  if (!L.keyed) leaf_key(L);
  app->cache.put(L.key, v);
}

// Pack buffers for GPU batches: pinned (gv_host_alloc), so the library reads
// them in place (direct H2D, or zero-copy for small batches) instead of
// staging pageable memory; recycled, so a block's pack neither page-faults a
// fresh allocation nor pays hipHostMalloc again.
gvh_app::PinBuf pin_get(gvh_app* app, size_t bytes) {
  {
    std::lock_guard<std::mutex> g(app->pin_mu);
    auto& v = app->pin_free;
    size_t best = v.size();
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].cap >= bytes && (best == v.size() || v[i].cap < v[best].cap)) best = i;
    if (best < v.size()) {
      gvh_app::PinBuf b = v[best];
      v.erase(v.begin() + (long)best);
      return b;
    }
  }
  gvh_app::PinBuf b;
  b.cap = std::max<size_t>(bytes, size_t(1) << 20);
  void* p = nullptr;
  if (app->gpu && gv_host_alloc(app->gpu, b.cap, &p) == GV_OK && p) {
    b.p = (uint8_t*)p;
    b.pinned = true;
  } else {
    b.p = (uint8_t*)malloc(b.cap);
    if (!b.p) throw std::bad_alloc();
  }
  return b;
}
void pin_put(gvh_app* app, gvh_app::PinBuf b) {
  if (!b.p) return;
  std::lock_guard<std::mutex> g(app->pin_mu);
  auto& v = app->pin_free;
  v.push_back(b);
  if (v.size() > 4) {                                 // keep the four largest
    size_t s = 0;
    for (size_t i = 1; i < v.size(); ++i)
      if (v[i].cap < v[s].cap) s = i;
    if (v[s].pinned) gv_host_free(app->gpu, v[s].p);
    else free(v[s].p);
    v.erase(v.begin() + (long)s);
  }
}

// One GPU batch of leaves: packed on the pool (batch_pack), verified under
// the GPU lock with no pool use (batch_run: safe on another thread while the
// pool runs a block's ante loop), verdicts written back (batch_finish).
struct GpuBatch {
  std::vector<Leaf*> miss;                     // secp256k1 leaves (the ed25519 ones appended by batch_finish)
  std::vector<Leaf*> ed;
  gvh_app::PinBuf buf;
  size_t m = 0;
  uint8_t *pub = nullptr, *sig = nullptr, *dig = nullptr, *ok = nullptr;
  uint32_t* slots = nullptr;                   // keyed: key-arena slot per leaf, UINT32_MAX = not resident
  bool split = false;                          // miss holds the secp256k1 leaves only, ed the ed25519 ones
  bool all_dig = false;                        // (split) every secp256k1 leaf has its digest
  bool msgs = false;                           // gpu_hash: sign bytes in blob/moff/mlen instead of dig
  uint8_t* blob = nullptr;
  uint64_t* moff = nullptr;
  uint32_t* mlen = nullptr;
  bool looked_up = false;                      // slots filled against arena generation `gen`
  uint64_t gen = 0;
  std::vector<uint8_t> epub, esig, eok, eblob;
  std::vector<uint64_t> eoff;
  std::vector<uint32_t> elen;
};

// Layout of the pinned buffer: pub33 | sig64 | dig32 | slots (u32) | ok, or
// when no leaf has its digest (gpu_hash plans): pub33 | sig64 | sign bytes
// (each distinct message once: a multisig's leaves share one) | off (u64) |
// len (u32) | slots | ok, for gv_verify_msgs*.  A batch mixing both kinds
// hashes the missing digests here.
// Keyed: every key is looked up in the app's slot map here, on the pool,
// under the shared key lock (the map only gains entries while the arena
// generation stays the same, so a slot found here is still valid when the
// batch runs unless the generation moved -- batch_run checks).
void batch_pack(gvh_app* app, GpuBatch& b) {
  size_t undig = 0;
  if (!b.split) {                              // mixed misses (resolve): one pass splits them
    size_t k = 0;
    for (Leaf* L : b.miss) {
      if (L->kind) {
        b.ed.push_back(L);
      } else {
        undig += L->has_dig ? 0 : 1;
        b.miss[k++] = L;
      }
    }
    b.miss.resize(k);
  } else if (!b.all_dig) {
    undig = b.miss.size();                     // gpu_hash plans: no secp256k1 leaf has a digest
  }
  const size_t m = b.m = b.miss.size();
  if (m) {
    b.msgs = undig == m;
    std::vector<uint64_t> src;                 // msgs: leaf k's message starts at moff[k]; src[k] = 1 if k copies it
    size_t blob_n = 0;
    if (b.msgs) {
      src.resize(m);
      const std::string* prev = nullptr;
      for (size_t k = 0; k < m; ++k) {
        const std::string* s = b.miss[k]->msg.get();
        src[k] = s != prev;
        if (s != prev) blob_n += s->size();
        prev = s;
      }
    }
    const size_t off_at = (m * 97 + blob_n + 7) & ~size_t(7);   // msgs: the u64 offsets
    const size_t body = b.msgs ? off_at + m * 12 : m * 129;
    const size_t slot_off = (body + 15) & ~size_t(15);
    b.buf = pin_get(app, slot_off + m * 4 + m + 16);
    b.pub = b.buf.p;
    b.sig = b.pub + m * 33;
    if (b.msgs) {
      b.blob = b.sig + m * 64;
      b.moff = (uint64_t*)(b.buf.p + off_at);
      b.mlen = (uint32_t*)(b.moff + m);
      uint64_t at = 0;
      for (size_t k = 0; k < m; ++k) {         // offsets in order; copies below, on the pool
        if (src[k] && k) at += b.mlen[k - 1];
        b.moff[k] = at;
        b.mlen[k] = (uint32_t)b.miss[k]->msg->size();
      }
    } else {
      b.dig = b.sig + m * 64;
    }
    b.slots = (uint32_t*)(b.buf.p + slot_off);
    b.ok = b.buf.p + slot_off + m * 4;
    std::shared_lock<std::shared_mutex> rk(app->key_mu);
    const bool look = app->keyed && app->gpu && gv_keys_generation(app->gpu) == app->key_gen;
    b.gen = app->key_gen;
    b.looked_up = look;
    auto& map = app->key_slots;
    parallel_for(app, m, [&](size_t k) {
      Leaf& L = *b.miss[k];
      memcpy(&b.pub[k * 33], L.pub.data(), 33);
      memcpy(&b.sig[k * 64], L.sig.data(), 64);
      if (b.msgs) {
        if (src[k]) memcpy(b.blob + b.moff[k], L.msg->data(), L.msg->size());
      } else {
        ensure_dig(L);
        memcpy(&b.dig[k * 32], L.dig.data(), 32);
      }
      if (look) {
        const uint32_t* v = map.find(L.pub.data());
        b.slots[k] = v ? *v : UINT32_MAX;
      }
    });
  }
  const size_t me = b.ed.size();
  if (me) {
    b.epub.resize(me * 32);
    b.esig.resize(me * 64);
    b.eok.resize(me);
    b.eoff.resize(me);
    b.elen.resize(me);
    for (size_t k = 0; k < me; ++k) {
      memcpy(&b.epub[k * 32], b.ed[k]->pub.data(), 32);
      memcpy(&b.esig[k * 64], b.ed[k]->sig.data(), 64);
      b.eoff[k] = b.eblob.size();
      b.elen[k] = (uint32_t)b.ed[k]->msg->size();
      b.eblob.insert(b.eblob.end(), b.ed[k]->msg->begin(), b.ed[k]->msg->end());
    }
  }
}

// The secp256k1 part of a batch (gpu_mu held).  Keyed: keys not yet in the
// context's key arena are parsed into it with ONE gv_keys_load (batches of
// at least key_load_min leaves -- a block; a smaller batch with an unknown
// key takes the pub33 path rather than wait on the key-table build), and the
// batch runs gv_verify_digests_keyed -- the same verdicts as the pub33 path
// (a key ParsePubKey rejects keeps a false slot), without the per-item
// decompression and Q-table build, on the 4-group ladder.  Any arena problem
// (cap reached, load error) falls back to the pub33 batch for this call.
// ticket: queue the batch (gv_submit_*) instead of verifying it; the caller
// waits for *ticket (gv_wait) before it reads b.ok.  A batch queued keyed
// stays valid across a later gv_keys_load / gv_keys_reset: the library runs
// the queued batches before it moves a slot.
int verify_secp(gvh_app* app, GpuBatch& b, uint64_t* ticket = nullptr) {
  const size_t m = b.m;
  auto plain = [&] {
    if (ticket)
      return b.msgs ? gv_submit_msgs(app->gpu, m, b.pub, b.sig, b.blob, b.moff, b.mlen, b.ok, ticket)
                    : gv_submit_digests(app->gpu, m, b.pub, b.sig, b.dig, b.ok, ticket);
    return b.msgs ? gv_verify_msgs(app->gpu, m, b.pub, b.sig, b.blob, b.moff, b.mlen, b.ok)
                  : gv_verify_digests(app->gpu, m, b.pub, b.sig, b.dig, b.ok);
  };
  if (!app->keyed) return plain();
  constexpr uint32_t kPending = 0x80000000u;      // map value of a key queued for this call's load
  std::unique_lock<std::shared_mutex> wk(app->key_mu);
  auto& map = app->key_slots;
  const uint64_t gen = gv_keys_generation(app->gpu);
  if (gen != app->key_gen) {                      // the arena was reset (here or by another user)
    map.clear();
    app->key_gen = gen;
  }
  if (!b.looked_up || b.gen != gen)               // packed against another arena: look up again
    for (size_t k = 0; k < m; ++k) {
      const uint32_t* v = map.find(b.pub + 33 * k);
      b.slots[k] = v ? *v : UINT32_MAX;
    }
  if (m < app->key_load_min) {                    // small batch (CheckTx window, per-tx ante)
    bool all = true;
    for (size_t k = 0; k < m && all; ++k) all = b.slots[k] != UINT32_MAX;
    if (!all) return plain();
  }
  std::vector<uint8_t> fresh;
  std::vector<std::array<uint8_t, 33>> fresh_keys;
  for (size_t k = 0; k < m; ++k) {
    if (b.slots[k] != UINT32_MAX) continue;
    std::array<uint8_t, 33> key;
    memcpy(key.data(), b.pub + 33 * k, 33);
    auto ins = map.emplace(key.data(), kPending + (uint32_t)fresh_keys.size());
    if (ins.second) {
      fresh.insert(fresh.end(), key.begin(), key.end());
      fresh_keys.push_back(key);
    }
    b.slots[k] = *ins.first;
  }
  if (!fresh_keys.empty()) {
    const size_t nf = fresh_keys.size();
    std::vector<uint32_t> got(nf);
    const bool room = gv_keys_count(app->gpu) + nf <= app->key_cap;
    if (!room || gv_keys_load(app->gpu, nf, fresh.data(), got.data()) != GV_OK) {
      if (!room) {                                  // start the arena over; this call takes the pub33 path
        gv_keys_reset(app->gpu);
        map.clear();
        app->key_gen = gv_keys_generation(app->gpu);
      } else {
        for (auto& key : fresh_keys) map.erase(key.data());
      }
      return plain();
    }
    for (size_t i = 0; i < nf; ++i) map.set(fresh_keys[i].data(), got[i]);
    for (size_t k = 0; k < m; ++k)
      if (b.slots[k] >= kPending) b.slots[k] = got[b.slots[k] - kPending];
  }
  if (ticket)
    return b.msgs ? gv_submit_msgs_keyed(app->gpu, m, b.slots, b.sig, b.blob, b.moff, b.mlen, b.ok, ticket)
                  : gv_submit_digests_keyed(app->gpu, m, b.slots, b.sig, b.dig, b.ok, ticket);
  return b.msgs ? gv_verify_msgs_keyed(app->gpu, m, b.slots, b.sig, b.blob, b.moff, b.mlen, b.ok)
                : gv_verify_digests_keyed(app->gpu, m, b.slots, b.sig, b.dig, b.ok);
}

// m ed25519 leaves (gpu_mu held): keyed against the context's ed25519 key
// arena when every key is resident, or when `load` (a commit's validator set,
// a block-sized batch) -- the missing keys are then loaded with one
// gv_ed_keys_load; otherwise, or on any arena problem, the unkeyed batch.
// Same verdicts either way (gv_verify_ed25519_msgs_keyed's contract).
int verify_ed(gvh_app* app, size_t m, const uint8_t* pub, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
              const uint32_t* len, uint8_t* ok, bool load) {
  if (!app->keyed) return gv_verify_ed25519_msgs(app->gpu, m, pub, sig, blob, off, len, ok);
  auto& map = app->ed_slots;
  const uint64_t gen = gv_ed_keys_generation(app->gpu);
  if (gen != app->ed_key_gen) {                   // the arena was reset (here or by another user)
    map.clear();
    app->ed_key_gen = gen;
  }
  std::vector<uint32_t> slots(m);
  std::vector<uint8_t> fresh;
  std::vector<std::array<uint8_t, 32>> fresh_keys;
  constexpr uint32_t kPending = 0x80000000u;
  for (size_t k = 0; k < m; ++k) {
    std::array<uint8_t, 32> key;
    memcpy(key.data(), pub + 32 * k, 32);
    if (const uint32_t* v = map.find(key.data())) { slots[k] = *v; continue; }
    if (!load) return gv_verify_ed25519_msgs(app->gpu, m, pub, sig, blob, off, len, ok);
    auto ins = map.emplace(key.data(), kPending + (uint32_t)fresh_keys.size());
    if (ins.second) {
      fresh.insert(fresh.end(), key.begin(), key.end());
      fresh_keys.push_back(key);
    }
    slots[k] = *ins.first;
  }
  if (!fresh_keys.empty()) {
    const size_t nf = fresh_keys.size();
    std::vector<uint32_t> got(nf);
    const bool room = gv_ed_keys_count(app->gpu) + nf <= GV_ED_KEY_CAP;
    if (!room || gv_ed_keys_load(app->gpu, nf, fresh.data(), got.data()) != GV_OK) {
      if (!room) {
        gv_ed_keys_reset(app->gpu);
        map.clear();
        app->ed_key_gen = gv_ed_keys_generation(app->gpu);
      } else {
        for (auto& key : fresh_keys) map.erase(key.data());
      }
      return gv_verify_ed25519_msgs(app->gpu, m, pub, sig, blob, off, len, ok);
    }
    for (size_t i = 0; i < nf; ++i) map.set(fresh_keys[i].data(), got[i]);
    for (size_t k = 0; k < m; ++k)
      if (slots[k] >= kPending) slots[k] = got[slots[k] - kPending];
  }
  return gv_verify_ed25519_msgs_keyed(app->gpu, m, slots.data(), sig, blob, off, len, ok);
}

int batch_run(gvh_app* app, GpuBatch& b) {
  if (!app->gpu) return GVH_ENOVERIFIER;
  std::lock_guard<std::mutex> g(app->gpu_mu);
  if (b.m && verify_secp(app, b) != GV_OK) return GVH_EDEVICE;
  const size_t me = b.ed.size();
  if (me && verify_ed(app, me, b.epub.data(), b.esig.data(), b.eblob.empty() ? nullptr : b.eblob.data(), b.eoff.data(),
                      b.elen.data(), b.eok.data(), me >= app->key_load_min) != GV_OK)
    return GVH_EDEVICE;
  return GVH_OK;
}

// A batch without ed25519 leaves queued on the library's asynchronous path:
// *ticket = 0 when there is nothing to wait for.
int batch_submit(gvh_app* app, GpuBatch& b, uint64_t* ticket) {
  *ticket = 0;
  if (!app->gpu) return GVH_ENOVERIFIER;
  std::lock_guard<std::mutex> g(app->gpu_mu);
  if (b.m && verify_secp(app, b, ticket) != GV_OK) return GVH_EDEVICE;
  return GVH_OK;
}
int batch_wait(gvh_app* app, uint64_t ticket) {
  if (!ticket) return GVH_OK;
  return gv_wait(app->gpu, ticket) == GV_OK ? GVH_OK : GVH_EDEVICE;
}

void batch_finish(gvh_app* app, GpuBatch& b, bool fill, uint32_t* gpu_leaves) {
  const size_t m = b.m, me = b.ed.size();
  app->st_gpu_calls += (m ? 1 : 0) + (me ? 1 : 0);
  app->st_gpu_leaves += m + me;
  parallel_for(app, m + me, [&](size_t k) {
    Leaf* L = k < m ? b.miss[k] : b.ed[k - m];
    const uint8_t v = k < m ? b.ok[k] : b.eok[k - m];
    L->verdict = v;
    if (fill) cache_insert(app, *L, v != 0);
  });
  if (gpu_leaves) *gpu_leaves += (uint32_t)(m + me);
  pin_put(app, b.buf);
  b.buf = gvh_app::PinBuf{};
}
void batch_drop(gvh_app* app, GpuBatch& b) {
  pin_put(app, b.buf);
  b.buf = gvh_app::PinBuf{};
}

// Resolve leaves: cache first, the misses in ONE GPU batch per key type.
int resolve(gvh_app* app, std::vector<Leaf*>& leaves, uint32_t* gpu_leaves, uint32_t* hits, bool all_miss = false,
            bool fill = true) {
  std::vector<Leaf*> miss;
  if (all_miss) {                                     // the caller already looked every leaf up
    miss.swap(leaves);
  } else if (leaves.size() >= 4096) {                        // big batches: lookups on the pool
    parallel_for(app, leaves.size(), [&](size_t i) {
      Leaf* L = leaves[i];
      if (L->verdict < 0) L->verdict = cache_lookup(app, *L);
    });
    for (Leaf* L : leaves)
      if (L->verdict < 0) miss.push_back(L);
    if (hits) *hits += (uint32_t)(leaves.size() - miss.size());
  } else {
    for (Leaf* L : leaves) {
      if (L->verdict >= 0) { if (hits) ++*hits; continue; }
      const int v = cache_lookup(app, *L);
      if (v >= 0) { L->verdict = v; if (hits) ++*hits; }
      else miss.push_back(L);
    }
  }
  if (!all_miss) app->st_hits += leaves.size() - miss.size();
  app->st_misses += miss.size();
  if (miss.empty()) return GVH_OK;
  if (!app->gpu) return GVH_ENOVERIFIER;
  const bool prof = getenv("GVH_PROFILE") != nullptr;
  double tr = prof ? prof_ms() : 0.0;
  auto rlap = [&](const char* what) {
    if (!prof) return;
    const double t = prof_ms();
    fprintf(stderr, "resolve %s %.3f ms\n", what, t - tr);
    tr = t;
  };
  GpuBatch b;
  b.miss.swap(miss);
  batch_pack(app, b);
  rlap("pack");
  if (batch_run(app, b) != GVH_OK) {
    batch_drop(app, b);
    return GVH_EDEVICE;
  }
  rlap("gv_verify");
  batch_finish(app, b, fill, gpu_leaves);
  rlap("put");
  return GVH_OK;
}

// The ante chain on one decoded tx (app->mu held by the caller).  memo: the
// PreVerifyTxs work for these bytes, or null.  Every memoised value is used
// only after checking that the state it was computed from is the state now.
int run_ante(gvh_app* app, const Tx& tx, Memo* memo, bool simulate, gvh_result* out) {
  const uint64_t wanted = tx.gas;
  // SetGasMeter (setup.go:67-76): infinite when simulating or at height 0
  GasMeter gm{!app->gas_limit && (simulate || app->height == 0), app->gas_limit ? app->gas_limit : tx.gas};
  uint32_t gpu_leaves = 0, hits = 0;
  // runTx runs the ante handler on a cache-wrapped context and writes it only
  // on success (baseapp/baseapp.go:553-578): a failed chain leaves no state.
  Account* set_pub[8];
  int n_set = 0;
  std::vector<Account*> set_pub_more;
  auto rollback = [&]() {
    for (int k = 0; k < n_set; ++k) { set_pub[k]->pub.clear(); set_pub[k]->info = nullptr; }
    for (Account* a : set_pub_more) { a->pub.clear(); a->info = nullptr; }
  };
  auto fail = [&](const SdkError& e) {
    rollback();
    copy_result(out, &e, gm.used, gpu_leaves, hits, wanted);
    return GVH_OK;
  };
  try {
    if (tx.nil_msg) throw Panic("runtime error: invalid memory address or nil pointer dereference");
    const auto& signers = tx.signers;
    const size_t ns = tx.sigs.size();
    // GetPubKeys(): amino-decode every tx-supplied pubkey (MustUnmarshal -> panic)
    std::vector<std::shared_ptr<const PubInfo>> local;
    const std::vector<std::shared_ptr<const PubInfo>>* tx_pk = nullptr;
    if (memo && memo->tx_pk.size() == ns) {
      if (memo->pk_panic >= 0) throw Panic(memo->pk_panic_msg);
      tx_pk = &memo->tx_pk;
    } else {
      local.resize(ns);
      for (size_t i = 0; i < ns; ++i)
        if (tx.sigs[i].pub.n) local[i] = app->pubs.get(tx.sigs[i].pub.p, tx.sigs[i].pub.n);
      tx_pk = &local;
    }
    // signer accounts, looked up once (PreVerifyTxs' lookups reused: account
    // entries are never removed, so a found pointer stays valid)
    Account* accs_small[8] = {};
    std::vector<Account*> accs_big;
    if (signers.size() > 8) accs_big.assign(signers.size(), nullptr);
    Account** accs = signers.size() > 8 ? accs_big.data() : accs_small;
    if (memo && memo->sacc.size() == signers.size())
      for (size_t i = 0; i < signers.size(); ++i) accs[i] = memo->sacc[i];
    auto acc_of = [&](size_t i) -> Account* {
      if (!accs[i]) accs[i] = find_account(app, signers[i]);
      return accs[i];
    };
    static const std::shared_ptr<const PubInfo> kSim = [] {
      auto p = std::make_shared<PubInfo>();
      p->raw = kSimPub;
      p->pk = decode_pubkey(kSimPub.data(), kSimPub.size());
      p->canon = kSimPub;
      p->addr = pubkey_address(p->pk);
      return std::shared_ptr<const PubInfo>(p);
    }();

    // KV-store gas (app->kv_gas): accounts and params are read through gaskv.
    const bool kv = app->kv_gas;
    auto acc_len = [](const Account& a) { return account_value_len(a.pub.size(), a.number, a.sequence); };
    auto acc_read = [&](const Account* a) {          // AccountKeeper.GetAccount (keeper/account.go:30-38)
      if (kv) kv_read(gm, a ? acc_len(*a) : 0);
    };
    auto acc_write = [&](const Account& a) {         // AccountKeeper.SetAccount (keeper/account.go:51-61)
      if (kv) kv_write(gm, acc_len(a));
    };
    auto params_gas = [&]() {                        // AccountKeeper.GetParams: five metered Gets
      if (!kv) return;
      for (uint64_t v : {kMaxMemoCharacters, app->sig_limit, kTxSizeCostPerByte, app->cost_ed, app->cost_secp})
        kv_read(gm, amino_json_u64_len(v));
    };

    // ---- ValidateMemoDecorator (x/auth/ante/basic.go:61-77)
    params_gas();
    if (tx.memo_len > kMaxMemoCharacters)
      return fail(wrap(kErrMemoTooLarge, "maximum number of characters is " + std::to_string(kMaxMemoCharacters) +
                                             " but received " + std::to_string(tx.memo_len) + " characters"));
    // ---- ConsumeTxSizeGasDecorator (basic.go:98-148)
    if (kv) {
      params_gas();
      gm.consume(kTxSizeCostPerByte * tx.raw.n, "txSize");
      if (simulate) {                                // a signature left empty: the size of a full one
        for (size_t i = 0; i < signers.size(); ++i) {
          if (i >= ns) throw Panic("runtime error: index out of range");
          if (tx.sigs[i].sig.n) continue;
          Account* acc = acc_of(i);
          acc_read(acc);
          const std::shared_ptr<const PubInfo> info = acc ? account_info(app, *acc) : nullptr;
          const PubInfo& pk = info ? *info : *kSim;
          // amino StdSignature{PubKey: pk.Bytes(), Signature: simSecp256k1Sig[:]} + 6
          uint64_t cost = 1 + uvarint_len(pk.canon.size()) + pk.canon.size() + 1 + 1 + 64 + 6;
          if (pk.pk.kind == PubKey::Multisig) cost *= app->sig_limit;
          gm.consume(kTxSizeCostPerByte * cost, "txSize");
        }
      }
    }

    // ---- SetPubKeyDecorator (sigverify.go:60-99)
    for (size_t i = 0; i < ns; ++i) {
      const PubInfo* pk = (*tx_pk)[i].get();
      if (!pk && !simulate) continue;                 // pubkey already set on the account
      if (i >= signers.size()) throw Panic("runtime error: index out of range");
      if (!simulate) {
        if (pk->pk.kind == PubKey::Nil) throw Panic("runtime error: invalid memory address or nil pointer dereference");
        if (!(signers[i].n == 20 && !memcmp(pk->addr.data(), signers[i].p, 20)))
          return fail(wrap(kErrInvalidPubKey, "pubKey does not match signer address " + acc_string(signers[i]) +
                                                  " with signer index: " + std::to_string(i)));
      }
      Account* acc = acc_of(i);
      acc_read(acc);                                  // GetSignerAcc (:83)
      if (!acc) return fail(wrap(kErrUnknownAddress, "account " + acc_string(signers[i]) + " does not exist"));
      if (acc->pub.empty()) {
        const auto& info = pk ? (*tx_pk)[i] : kSim;
        acc->pub = info->canon;
        acc->info = info->canon == info->raw ? info : nullptr;
        if (n_set < 8) set_pub[n_set++] = acc;
        else set_pub_more.push_back(acc);
        acc_write(*acc);                              // SetAccount (:95)
      }
    }
    // ---- ValidateSigCountDecorator (sigverify.go:275-294)
    params_gas();
    {
      uint64_t count = 0;
      for (size_t i = 0; i < ns; ++i) {
        count += (*tx_pk)[i] ? (uint64_t)(*tx_pk)[i]->subkeys : 1;   // CountSubKeys(nil) -> 1
        if (count > app->sig_limit)
          return fail(wrap(kErrTooManySignatures,
                           "signatures: " + std::to_string(count) + ", limit: " + std::to_string(app->sig_limit)));
      }
    }
    // ---- DeductFeeDecorator (x/auth/ante/fee.go:84-108): the fee payer's
    // account read.  (A nonzero fee's bank transfer is not modelled: the
    // mirror keeps no balances.)
    if (kv) {
      Account* payer = signers.empty() ? nullptr : acc_of(0);     // StdTx.FeePayer() = GetSigners()[0]
      acc_read(payer);
      if (!payer)
        return fail(wrap(kErrUnknownAddress, "fee payer address: " +
                                                 (signers.empty() ? std::string() : acc_string(signers[0])) +
                                                 " does not exist"));
    }
    // ---- SigGasConsumeDecorator (sigverify.go:117-153)
    params_gas();
    for (size_t i = 0; i < ns; ++i) {
      if (i >= signers.size()) throw Panic("runtime error: index out of range");
      Account* acc = acc_of(i);
      acc_read(acc);                                  // GetSignerAcc (:131)
      if (!acc) return fail(wrap(kErrUnknownAddress, "account " + acc_string(signers[i]) + " does not exist"));
      std::shared_ptr<const PubInfo> pk = account_info(app, *acc);
      if (!pk) {
        if (!simulate) return fail(wrap(kErrInvalidPubKey, "unrecognized public key type: <nil>"));
        pk = kSim;
      }
      if (memo && i < memo->plans.size()) {
        const SignerPlan& mp = memo->plans[i];
        if (mp.ok && mp.gas_status == 0 && (mp.pub == pk || mp.pub->canon == acc->pub) && gm.fits(mp.gas)) {
          gm.used += mp.gas;                          // the same charge, computed in PreVerifyTxs
          continue;
        }
      }
      SdkError e;
      if (!consume_sig_gas(gm, tx.sigs[i].sig, pk->pk, app, &e)) return fail(e);
    }
    // ---- BatchSigVerificationDecorator (replaces sigverify.go:170-216)
    // Gather every signer's leaves up to the first signer the reference loop
    // would stop at (no gas: the look-ahead reads the state without a
    // meter), answer all leaves at once, then walk the signers in the
    // reference's order, charging each signer's account read only when the
    // loop gets there: the same gas as verifying one signer at a time.
    if (!app->recheck) {
      if (ns != signers.size())
        return fail(wrap(kErrUnauthorized, "invalid number of signer;  expected: " + std::to_string(signers.size()) +
                                               ", got " + std::to_string(ns)));
      std::vector<SignerPlan> fresh;                 // plans rebuilt here (a prediction missed)
      SignerPlan* plans_small[8];
      std::vector<SignerPlan*> plans_big;
      size_t np = 0;
      for (size_t i = 0; i < ns && !simulate; ++i) {
        Account* acc = acc_of(i);
        if (!acc || acc->pub.empty()) break;          // the walk reports it at signer i
        const uint64_t accnum = app->height == 0 ? 0 : acc->number;
        SignerPlan* p = nullptr;
        if (memo && i < memo->plans.size()) {
          SignerPlan& mp = memo->plans[i];
          if (mp.ok && mp.accnum == accnum && mp.seq == acc->sequence &&
              (mp.pub == acc->info || mp.pub->canon == acc->pub)) {
            p = &mp;
            app->st_memo += 1;
          }
        }
        if (!p) {
          if (fresh.capacity() == 0) fresh.reserve(ns);   // pointers into it must stay valid
          fresh.emplace_back();
          p = &fresh.back();
          make_plan(*p, app, tx, i, account_info(app, *acc), accnum, acc->sequence, app->chain_json);
        }
        if (np < 8) plans_small[np] = p;
        else plans_big.push_back(p);
        ++np;
      }
      auto plan_at = [&](size_t k) { return k < 8 ? plans_small[k] : plans_big[k - 8]; };
      bool all_resolved = true;
      for (size_t k = 0; k < np; ++k) all_resolved = all_resolved && plan_at(k)->resolved;
      if (all_resolved) {
        for (size_t k = 0; k < np; ++k) hits += (uint32_t)plan_at(k)->leaves.size();
      } else {
        std::vector<Leaf*> leaves;
        for (size_t k = 0; k < np; ++k)
          for (Leaf& L : plan_at(k)->leaves) leaves.push_back(&L);
        if (!leaves.empty()) {
          const int rc = resolve(app, leaves, &gpu_leaves, &hits);
          if (rc != GVH_OK) { rollback(); return rc; }
        }
      }
      for (size_t i = 0; i < ns; ++i) {               // the reference loop (sigverify.go:194-213)
        Account* acc = acc_of(i);
        acc_read(acc);                                // GetSignerAcc (:195)
        if (!acc) return fail(wrap(kErrUnknownAddress, "account " + acc_string(signers[i]) + " does not exist"));
        if (!simulate && acc->pub.empty()) return fail(wrap(kErrInvalidPubKey, "pubkey on account is not set"));
        if (simulate) continue;
        if (!eval(plan_at(i)->node, plan_at(i)->leaves))
          return fail(wrap(kErrUnauthorized, "signature verification failed; verify correct account sequence and chain-id"));
      }
    }
    // ---- IncrementSequenceDecorator (sigverify.go:237-259)
    if (!app->recheck || simulate) {
      for (size_t i = 0; i < signers.size(); ++i) {
        Account* acc = acc_of(i);
        acc_read(acc);
        if (!acc) throw Panic("account not found");
        acc->sequence += 1;
        acc_write(*acc);
      }
    }
  } catch (const Panic& p) {
    return fail(wrap(kErrPanic, p.what()));
  } catch (const OutOfGas& o) {
    return fail(wrap(kErrOutOfGas, std::string("out of gas in location: ") + o.descriptor + "; gasWanted: " +
                                       std::to_string(wanted) + ", gasUsed: " + std::to_string(gm.used)));
  }
  copy_result(out, nullptr, gm.used, gpu_leaves, hits, wanted);
  return GVH_OK;
}

int ante_memo(gvh_app* app, Memo* m, bool simulate, gvh_result* out) {
  if (!m->tx) {
    SdkError err = wrap(kErrTxDecode, m->decode_err);
    copy_result(out, &err, 0, 0, 0, 0);
    return GVH_OK;
  }
  std::lock_guard<std::mutex> lk(app->mu);
  return run_ante(app, *m->tx, m, simulate, out);
}

// ante on raw bytes: decode (or reuse the memo), then the chain.
int ante_bytes(gvh_app* app, const uint8_t* p, size_t n, bool simulate, gvh_result* out) {
  std::shared_ptr<Memo> m = app->memo.find(p, n);
  if (m) return ante_memo(app, m.get(), simulate, out);
  std::shared_ptr<const Tx> tx;
  try {
    tx = decode_tx(p, n, false);
  } catch (const AminoErr& e) {
    SdkError err = wrap(kErrTxDecode, e.what());
    copy_result(out, &err, 0, 0, 0, 0);
    return GVH_OK;
  }
  std::lock_guard<std::mutex> lk(app->mu);
  return run_ante(app, *tx, nullptr, simulate, out);
}

// Drop a block's memos on the pool.  Every worker frees what it allocated --
// first the plans it built, then the memos it decoded -- so each free returns
// to the freeing thread's own malloc arena: frees spread over the pool at
// random contend on the other arenas' locks (measured: 3.3 ms vs ~0.3 ms for a
// 10k-tx multisig block on 16 threads).
// Owners are read before any worker starts moving elements out (a worker must
// not read an element another worker is resetting); part p of np releases the
// memos whose owner is p modulo np.
std::vector<int16_t> memo_owners(const std::vector<std::shared_ptr<Memo>>& memos) {
  std::vector<int16_t> own(memos.size());
  for (size_t i = 0; i < memos.size(); ++i) own[i] = memos[i] ? memos[i]->owner : (int16_t)-1;
  return own;
}
void release_part(gvh_app* app, std::vector<std::shared_ptr<Memo>>& memos, const std::vector<int16_t>& own, int p,
                  int np) {
  for (size_t i = 0; i < memos.size(); ++i) {
    if (own[i] < 0 || own[i] % np != p) continue;
    std::shared_ptr<Memo>& m = memos[i];
    if (m.use_count() == 1) memo_put(app, own[i], std::move(m));   // unshared: back to its worker's pool
    else m.reset();                                                // the memo table's: just dropped
  }
}
void release_memos(gvh_app* app, std::vector<std::shared_ptr<Memo>>& memos) {
  const std::vector<int16_t> own = memo_owners(memos);
  parallel_workers(app, [&](int w, int nw) { release_part(app, memos, own, w, nw); });
  memos.clear();
}

// PreVerifyTxs in three parts, so a pipelined replay (deliver_blocks) can run
// one block's GPU batch on another thread while the pool delivers the block
// before it:
//   pre_front  decode, sequence prediction and plans (app lock held while the
//              state is read), then the misses packed into one batch
//   batch_run  the GPU batch (no pool, no app lock)
//   pre_back   verdicts written back, plans marked resolved, memos kept or released
// carry_from: the epoch of a block pre-verified but not yet delivered, whose
// effects (sequence increments, SetPubKey) the prediction adds to the state
// (0: none -- every block delivered).
struct PreState {
  std::vector<std::shared_ptr<Memo>> memos;
  std::vector<SignerPlan*> plans;
  GpuBatch batch;
  bool has_batch = false, keep = false;
  uint64_t epoch = 0;
  size_t n_all = 0;
};

void pre_front(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, bool keep,
               uint64_t carry_from, PreState& ps) {
  const bool prof = getenv("GVH_PROFILE") != nullptr;
  double T0 = prof ? prof_ms() : 0.0;
  auto lap = [&](const char* what) {
    if (!prof) return;
    const double t = prof_ms();
    fprintf(stderr, "preverify %s %.3f ms\n", what, t - T0);
    T0 = t;
  };
  ps.keep = keep;
  std::unique_lock<std::mutex> lk(app->mu);
  const std::string chain_json = app->chain_json;
  const bool gpu_hash = !keep && app->gpu_hash && app->gpu && app->cache.size() == 0;
  // (1) parallel: decode (sharing an earlier decode of the same bytes),
  // GetPubKeys' tx-supplied keys, the signers' accounts
  std::vector<std::shared_ptr<Memo>>& memos = ps.memos;
  memos.assign(ntx, nullptr);
  // stage (2)'s signer partition, decided here: part_mask[t] = the parts tx t touches
  const int parts = ntx >= 2048 ? std::max(1, std::min(64, app->threads)) : 1;
  auto part_of = [&](const Account* a) { return (int)(((uintptr_t)a >> 4) % (uintptr_t)parts); };
  std::vector<uint64_t> part_mask(ntx, 0);
  parallel_for_w(app, ntx, [&](size_t t, int w) {
    // a fresh Memo every time (an earlier one may be in use by an ante run)
    auto m = memo_get(app, w);
    m->owner = (int16_t)w;
    auto old = keep ? app->memo.find(txs[t], lens[t]) : nullptr;
    if (old) m->tx = old->tx;
    else {
      try {
        m->tx = decode_tx(txs[t], lens[t], keep, tx_get(app, w));
      } catch (const AminoErr& e) {
        m->decode_err = e.what();
      }
    }
    if (m->tx) {
      const Tx& tx = *m->tx;
      m->sacc.resize(tx.signers.size());
      uint64_t mask = 0;
      for (size_t i = 0; i < tx.signers.size(); ++i) {
        m->sacc[i] = find_account(app, tx.signers[i]);
        if (m->sacc[i]) mask |= uint64_t(1) << part_of(m->sacc[i]);
      }
      part_mask[t] = mask;
      m->tx_pk.resize(tx.sigs.size());
      for (size_t i = 0; i < tx.sigs.size(); ++i) {
        const Span pb = tx.sigs[i].pub;
        if (!pb.n) continue;
        // the signer's account already holds these exact (canonical) bytes:
        // its decoded key is the one GetPubKeys would decode (no table lookup)
        const Account* a = i < m->sacc.size() ? m->sacc[i] : nullptr;
        if (a && a->info && a->pub.size() == pb.n && !memcmp(a->pub.data(), pb.p, pb.n)) {
          m->tx_pk[i] = a->info;
          continue;
        }
        try {
          m->tx_pk[i] = app->pubs.get(pb.p, pb.n);
        } catch (const Panic& e) {
          m->pk_panic = (int)i;
          m->pk_panic_msg = e.what();
          break;
        }
      }
      m->plans.resize(tx.sigs.size());
    }
    memos[t] = std::move(m);
  });
  lap("decode");
  // (2) sequence prediction = a per-signer prefix count in block order (plus
  // the carried block's count); signers are hash-partitioned over the pool,
  // each part scanning the block in order for its own signers (every account
  // is touched by one part only).  The predicted key is the account's, else
  // the one an earlier SetPubKey (this block or the carried one) stores, else
  // the tx-supplied one.
  struct Job {
    uint32_t t, signer;
    uint64_t accnum, seq;
    SignerPlan* plan;
    std::shared_ptr<const PubInfo> pub;       // the account's key after SetPubKey
  };
  std::vector<Job> jobs;
  {
    const uint64_t epoch = ps.epoch = ++app->bump_epoch;
    const uint64_t prev = carry_from;
    auto touch = [&](Account* acc) {
      if (acc->bump_epoch == epoch) return;
      const bool carry = prev && acc->own_epoch == prev;
      acc->bump_epoch = epoch;
      acc->bump = carry ? acc->own : 0;
      acc->pred_info = carry ? acc->own_info : nullptr;
      acc->own_epoch = epoch;
      acc->own = 0;
      acc->own_info = nullptr;
    };
    std::vector<std::vector<Job>> pj(parts);
    parallel_parts(app, parts, [&](int part) {
      std::vector<Job>& out = pj[part];
      out.reserve(ntx / parts + 16);
      for (size_t t = 0; t < ntx; ++t) {
        if (!(part_mask[t] >> part & 1)) continue;
        Memo& m = *memos[t];
        if (!m.tx || m.tx->nil_msg || m.pk_panic >= 0) continue;
        const Tx& tx = *m.tx;
        for (size_t i = 0; i < tx.sigs.size() && i < tx.signers.size(); ++i) {
          Account* acc = m.sacc[i];
          if (!acc || part_of(acc) != part) continue;
          touch(acc);
          std::shared_ptr<const PubInfo> pub;
          try {
            pub = account_info(app, *acc);
          } catch (const Panic&) {
            continue;
          }
          if (!pub) {
            pub = acc->pred_info;
            if (!pub && m.tx_pk[i]) {               // SetPubKey will store the tx-supplied key
              pub = m.tx_pk[i];
              acc->pred_info = acc->own_info = pub;
            }
          }
          if (!pub) continue;
          out.push_back(Job{(uint32_t)t, (uint32_t)i, app->height == 0 ? 0 : acc->number, acc->sequence + acc->bump,
                            &m.plans[i], std::move(pub)});
        }
        for (Account* acc : m.sacc)                    // every signer's sequence moves if the tx passes
          if (acc && part_of(acc) == part) {
            touch(acc);
            acc->bump += 1;
            acc->own += 1;
          }
      }
    });
    size_t tot = 0;
    for (auto& v : pj) tot += v.size();
    jobs.reserve(tot);
    for (auto& v : pj)
      for (auto& j : v) jobs.push_back(std::move(j));
  }
  lap("jobs");
  // (3) parallel: gas charge, sign bytes, leaves, cache keys + lookups; the
  // misses collect per worker
  // (secp256k1 and ed25519 misses apart, so batch_pack need not walk the leaves)
  std::vector<std::vector<Leaf*>> wmiss(std::max(1, app->threads)), wed(std::max(1, app->threads));
  std::atomic<size_t> n_leaf{0};
  parallel_for_w(app, jobs.size(), [&](size_t k, int w) {
    Job& j = jobs[k];
    Memo& m = *memos[j.t];
    j.plan->owner = (int16_t)w;
    try {
      make_plan(*j.plan, app, *m.tx, j.signer, j.pub, j.accnum, j.seq, chain_json, gpu_hash);
    } catch (const Panic&) {
      j.plan->ok = false;                               // malformed: the ante chain will report it
      return;
    }
    for (Leaf& L : j.plan->leaves) {
      if (L.verdict < 0) L.verdict = cache_lookup(app, L);
      if (L.verdict < 0) (L.kind ? wed[w] : wmiss[w]).push_back(&L);
    }
    n_leaf.fetch_add(j.plan->leaves.size(), std::memory_order_relaxed);
  });
  ps.n_all = n_leaf.load();
  lap("plans");
  lk.unlock();
  ps.plans.resize(jobs.size());
  for (size_t k = 0; k < jobs.size(); ++k) ps.plans[k] = jobs[k].plan;
  std::vector<Leaf*>& miss = ps.batch.miss;
  {
    size_t nm = 0;
    for (auto& v : wmiss) nm += v.size();
    miss.reserve(nm);
    for (auto& v : wmiss) miss.insert(miss.end(), v.begin(), v.end());
    for (auto& v : wed) ps.batch.ed.insert(ps.batch.ed.end(), v.begin(), v.end());
    ps.batch.split = true;
    ps.batch.all_dig = !gpu_hash;                    // fresh plans: digests exactly when not gpu_hash
  }
  app->st_hits += ps.n_all - miss.size() - ps.batch.ed.size();
  app->st_misses += miss.size() + ps.batch.ed.size();
  // (4) the misses packed for one GPU batch (pinned buffer, key slots looked up)
  if (!miss.empty() || !ps.batch.ed.empty()) {
    ps.has_batch = true;
    if (app->gpu) batch_pack(app, ps.batch);
  }
  lap("pack");
}

// The batch of a pre_front, timed into st_gpu_ns.
int pre_gpu(gvh_app* app, PreState& ps) {
  if (!ps.has_batch) return GVH_OK;
  const auto tg = std::chrono::steady_clock::now();
  const int rc = batch_run(app, ps.batch);
  app->st_gpu_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tg).count();
  return rc;
}

// rc: the batch's result.  A block being delivered (keep == false) reads the
// cache (txs seen by CheckTx) but does not fill it: its verdicts are used
// once, from the memos.
void pre_back(gvh_app* app, PreState& ps, int rc, size_t* n_leaves, std::vector<std::shared_ptr<Memo>>* memos_out) {
  uint32_t gpu_leaves = 0;
  if (ps.has_batch) {
    if (rc == GVH_OK) batch_finish(app, ps.batch, ps.keep, &gpu_leaves);
    else batch_drop(app, ps.batch);
  }
  if (rc == GVH_OK)
    parallel_for(app, ps.plans.size(), [&](size_t k) { ps.plans[k]->resolved = ps.plans[k]->ok; });
  if (ps.keep)
    for (auto& m : ps.memos) app->memo.put(m);
  if (n_leaves) *n_leaves = gpu_leaves;
  if (memos_out) *memos_out = std::move(ps.memos);
  else release_memos(app, ps.memos);
}

// PreVerifyTxs.  Returns the memos (one per tx, in order).  The app lock is
// held while the block's state is read (decode, sequence prediction, plans)
// and released for the GPU batch.
int preverify(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, size_t* n_leaves,
              std::vector<std::shared_ptr<Memo>>* memos_out, bool keep) {
  PreState ps;
  pre_front(app, ntx, txs, lens, keep, 0, ps);
  const int rc = ps.has_batch && !app->gpu ? GVH_ENOVERIFIER : pre_gpu(app, ps);
  pre_back(app, ps, rc, n_leaves, memos_out);
  return rc;
}

}  // namespace

extern "C" {

gvh_app* gvh_app_new(gv_ctx* gpu) {
  gvh_app* a = new gvh_app();
  a->gpu = gpu;
  return a;
}
void gvh_app_free(gvh_app* app) { delete app; }

void gvh_set_params(gvh_app* app, uint64_t lim, uint64_t cs, uint64_t ce) {
  std::lock_guard<std::mutex> lk(app->mu);
  app->sig_limit = lim;
  app->cost_secp = cs;
  app->cost_ed = ce;
}
void gvh_set_gas_model(gvh_app* app, int kv_gas) {
  std::lock_guard<std::mutex> lk(app->mu);
  app->kv_gas = kv_gas != 0;
}
void gvh_set_context(gvh_app* app, const char* chain_id, int64_t height, int recheck, uint64_t gas_limit) {
  std::lock_guard<std::mutex> lk(app->mu);
  app->chain_id = chain_id ? chain_id : "";
  app->chain_json = go_json_string(app->chain_id);
  app->height = height;
  app->recheck = recheck != 0;
  app->gas_limit = gas_limit;
}

int gvh_set_account(gvh_app* app, const uint8_t addr20[20], uint64_t num, uint64_t seq, const uint8_t* pub,
                    size_t pub_len) {
  if (!app || !addr20) return GVH_EINVAL;
  Addr a;
  memcpy(a.data(), addr20, 20);
  Account acc;
  acc.number = num;
  acc.sequence = seq;
  if (pub && pub_len) acc.pub.assign(pub, pub + pub_len);      // info decoded on first use
  std::lock_guard<std::mutex> lk(app->mu);
  app->accounts.get_or_insert(a) = acc;
  return GVH_OK;
}
int gvh_get_account(gvh_app* app, const uint8_t addr20[20], uint64_t* num, uint64_t* seq, uint8_t* pub_out,
                    size_t* pub_len) {
  Addr a;
  memcpy(a.data(), addr20, 20);
  std::lock_guard<std::mutex> lk(app->mu);
  Account* found = app->accounts.find(a.data());
  if (!found) return 0;
  if (num) *num = found->number;
  if (seq) *seq = found->sequence;
  if (pub_len) *pub_len = found->pub.size();
  if (pub_out && !found->pub.empty()) memcpy(pub_out, found->pub.data(), std::min<size_t>(512, found->pub.size()));
  return 1;
}

int gvh_ante(gvh_app* app, const uint8_t* tx, size_t tx_len, int simulate, gvh_result* out) {
  if (!app || (!tx && tx_len) || !out) return GVH_EINVAL;
  return ante_bytes(app, tx, tx_len, simulate != 0, out);
}

int gvh_preverify(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, size_t* n_leaves) {
  if (!app || (ntx && (!txs || !lens))) return GVH_EINVAL;
  return preverify(app, ntx, txs, lens, n_leaves, nullptr, true);
}

}  // extern "C"

namespace {

// The DeliverTx ante loop of a pre-verified block.  out and/or codes receive
// the results.  A tx's ante chain reads and writes only its signers'
// accounts (SetPubKey, IncrementSequence); when every tx has at most one
// signer, txs of different accounts are independent, so the loop runs as
// per-account chains in parallel (block order kept within each account) --
// the same results and final state as the serial loop.  Otherwise serial.
int deliver_memos(gvh_app* app, std::vector<std::shared_ptr<Memo>>& memos, gvh_result* out, uint32_t* codes) {
  const size_t ntx = memos.size();
  bool single = true;
  for (auto& m : memos)
    if (m->tx && m->tx->signers.size() > 1) { single = false; break; }
  auto one = [&](size_t t, gvh_result* r) {
    Memo* m = memos[t].get();
    if (!m->tx) {
      SdkError err = wrap(kErrTxDecode, m->decode_err);
      copy_result(r, &err, 0, 0, 0, 0);
      return GVH_OK;
    }
    return run_ante(app, *m->tx, m, false, r);
  };
  std::lock_guard<std::mutex> lk(app->mu);
  if (!single || ntx < 1024 || app->threads <= 1) {
    gvh_result tmp;
    for (size_t t = 0; t < ntx; ++t) {
      gvh_result* r = out ? &out[t] : &tmp;
      const int rc = one(t, r);
      if (rc != GVH_OK) return rc;
      if (codes) codes[t] = r->code;
    }
    return GVH_OK;
  }
  const int parts = app->threads;
  std::vector<std::vector<uint32_t>> idx(parts);
  for (size_t t = 0; t < ntx; ++t) {
    const Tx* tx = memos[t]->tx.get();
    int p = 0;
    if (tx && !tx->signers.empty() && tx->signers[0].n == 20) {
      const uint8_t* a = tx->signers[0].p;
      p = (int)((a[0] ^ a[7] ^ a[19]) % (unsigned)parts);
    }
    idx[p].push_back((uint32_t)t);
  }
  std::atomic<int> err{GVH_OK};
  parallel_parts(app, parts, [&](int p) {
    gvh_result tmp;
    for (uint32_t t : idx[p]) {
      if (err.load(std::memory_order_relaxed) != GVH_OK) return;
      gvh_result* r = out ? &out[t] : &tmp;
      const int rc = one(t, r);
      if (rc != GVH_OK) { err = rc; return; }
      if (codes) codes[t] = r->code;
    }
  });
  return err.load();
}

// One block: PreVerifyTxs, then the DeliverTx loop.  The previous block's
// memos (defer_release) go back to the worker pools while this block's GPU
// batch runs (the pool is otherwise idle then), and this block's wait for the
// next call.
int deliver_block(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, gvh_result* out,
                  uint32_t* codes) {
  std::vector<std::shared_ptr<Memo>> memos, stale;
  {
    std::lock_guard<std::mutex> g(app->deferred_mu);
    stale.swap(app->deferred);
  }
  const bool prof = getenv("GVH_PROFILE") != nullptr;
  const double p0 = prof ? prof_ms() : 0.0;
  const auto t0 = std::chrono::steady_clock::now();
  int rc;
  {
    PreState ps;
    pre_front(app, ntx, txs, lens, false, 0, ps);
    if (ps.has_batch && !app->gpu) {
      rc = GVH_ENOVERIFIER;
    } else if (ps.has_batch && !stale.empty() && app->threads > 1) {
      // the caller (worker 0) runs the batch, workers 1.. release the memos
      const std::vector<int16_t> own = memo_owners(stale);
      int rg = GVH_OK;
      parallel_workers(app, [&](int w, int nw) {
        if (w == 0) rg = pre_gpu(app, ps);
        else release_part(app, stale, own, w - 1, nw - 1);
      });
      stale.clear();
      rc = rg;
    } else {
      rc = pre_gpu(app, ps);
    }
    release_memos(app, stale);
    pre_back(app, ps, rc, nullptr, &memos);
  }
  const auto t1 = std::chrono::steady_clock::now();
  const double p1 = prof ? prof_ms() : 0.0;
  app->st_pre_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
  if (rc != GVH_OK) {
    release_memos(app, memos);
    return rc;
  }
  rc = deliver_memos(app, memos, out, codes);
  const auto t2 = std::chrono::steady_clock::now();
  const double p2 = prof ? prof_ms() : 0.0;
  app->st_loop_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
  if (app->defer_release) {
    std::lock_guard<std::mutex> g(app->deferred_mu);
    if (app->deferred.empty()) app->deferred.swap(memos);
  }
  release_memos(app, memos);                        // not deferred (option off, or another call's memos wait)
  if (prof)
    fprintf(stderr, "deliver preverify %.3f ms loop %.3f ms release %.3f ms\n", p1 - p0, p2 - p1, prof_ms() - p2);
  return rc;
}

// A run of consecutive blocks (block sync / replay: the blocks are known
// ahead of their delivery), pipelined: block b+1 is pre-verified -- its
// prediction carrying block b's sequence increments and SetPubKeys -- and its
// GPU batch runs on a helper thread while the pool delivers block b.  Results
// and final state are those of delivering the blocks one by one (a carried
// prediction that turns out wrong is a memo miss: the ante run rebuilds the
// plan from the state and verifies it, never a different verdict).
int deliver_blocks(gvh_app* app, size_t nb, const size_t* bn, const uint8_t* const* txs, const size_t* lens,
                   uint32_t* codes) {
  if (nb == 0) return GVH_OK;
  auto ns_since = [](std::chrono::steady_clock::time_point t) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count();
  };
  const bool prof = getenv("GVH_PROFILE") != nullptr;
  PreState cur, nxt;
  auto t0 = std::chrono::steady_clock::now();
  pre_front(app, bn[0], txs, lens, false, 0, cur);
  int rc = cur.has_batch && !app->gpu ? GVH_ENOVERIFIER : pre_gpu(app, cur);
  std::vector<std::shared_ptr<Memo>> memos;
  pre_back(app, cur, rc, nullptr, &memos);
  app->st_pre_ns += ns_since(t0);
  if (rc != GVH_OK) {
    release_memos(app, memos);
    return rc;
  }
  size_t off = 0;
  for (size_t b = 0; b < nb; ++b) {
    const bool more = b + 1 < nb;
    std::future<int> gpu;
    uint64_t ticket = 0;                              // block b+1's queued batch
    if (more) {
      const auto tp = std::chrono::steady_clock::now();
      nxt = PreState{};
      pre_front(app, bn[b + 1], txs + off + bn[b], lens + off + bn[b], false, cur.epoch, nxt);
      if (nxt.has_batch) {
        if (!app->gpu) {
          gpu = std::async(std::launch::deferred, [] { return (int)GVH_ENOVERIFIER; });
        } else if (app->async_blocks && nxt.batch.ed.empty()) {
          // queued on the library's asynchronous path: it runs while this
          // thread and the pool deliver block b (gv_wait below)
          const auto tg = std::chrono::steady_clock::now();
          const int rs = batch_submit(app, nxt.batch, &ticket);
          app->st_gpu_ns += ns_since(tg);
          if (rs != GVH_OK) gpu = std::async(std::launch::deferred, [rs] { return rs; });
        } else {
          gpu = std::async(std::launch::async, [app, &nxt] { return pre_gpu(app, nxt); });
        }
      }
      app->st_pre_ns += ns_since(tp);
      if (prof) fprintf(stderr, "blocks %zu: front %.3f ms\n", b + 1, ns_since(tp) / 1e6);
    }
    const auto tl = std::chrono::steady_clock::now();
    rc = deliver_memos(app, memos, nullptr, codes + off);
    app->st_loop_ns += ns_since(tl);
    release_memos(app, memos);
    if (prof) fprintf(stderr, "blocks %zu: loop+release %.3f ms\n", b, ns_since(tl) / 1e6);
    if (!more) break;
    const auto tw = std::chrono::steady_clock::now();
    int rg = gpu.valid() ? gpu.get() : GVH_OK;        // always joined before nxt goes away
    if (ticket) {
      const auto tg = std::chrono::steady_clock::now();
      rg = batch_wait(app, ticket);
      app->st_gpu_ns += ns_since(tg);
    }
    pre_back(app, nxt, rg, nullptr, &memos);
    if (prof) fprintf(stderr, "blocks %zu: gpu wait + back %.3f ms\n", b + 1, ns_since(tw) / 1e6);
    if (rc == GVH_OK) rc = rg;
    if (rc != GVH_OK) {
      release_memos(app, memos);
      return rc;
    }
    off += bn[b];
    cur.epoch = nxt.epoch;
  }
  return rc;
}

}  // namespace

extern "C" {

int gvh_deliver_block(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, gvh_result* out) {
  if (!app || (ntx && (!txs || !lens || !out))) return GVH_EINVAL;
  return deliver_block(app, ntx, txs, lens, out, nullptr);
}

int gvh_deliver_block_codes(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens,
                            uint32_t* codes) {
  if (!app || (ntx && (!txs || !lens || !codes))) return GVH_EINVAL;
  return deliver_block(app, ntx, txs, lens, nullptr, codes);
}

int gvh_deliver_blocks(gvh_app* app, size_t n_blocks, const size_t* block_ntx, const uint8_t* const* txs,
                       const size_t* lens, uint32_t* codes) {
  if (!app || (n_blocks && !block_ntx)) return GVH_EINVAL;
  size_t ntx = 0;
  for (size_t b = 0; b < n_blocks; ++b) ntx += block_ntx[b];
  if (ntx && (!txs || !lens || !codes)) return GVH_EINVAL;
  return deliver_blocks(app, n_blocks, block_ntx, txs, lens, codes);
}

int gvh_deliver_gentxs(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, gvh_result* out,
                       size_t* first_failed) {
  if (!app) return GVH_EINVAL;
  int64_t h;
  uint64_t gl;
  {
    std::lock_guard<std::mutex> lk(app->mu);
    h = app->height;
    gl = app->gas_limit;
    app->height = 0;                                  // InitChain context: genesis height, infinite gas
    app->gas_limit = 0;
  }
  const int rc = gvh_deliver_block(app, ntx, txs, lens, out);
  {
    std::lock_guard<std::mutex> lk(app->mu);
    app->height = h;
    app->gas_limit = gl;
  }
  if (first_failed) {
    *first_failed = ntx;
    if (rc == GVH_OK)
      for (size_t t = 0; t < ntx; ++t)
        if (out[t].code) { *first_failed = t; break; }
  }
  return rc;
}

void gvh_set_window(gvh_app* app, size_t max_txs, int64_t max_wait_us) {
  std::lock_guard<std::mutex> lk(app->window.m);
  app->window.max_txs = std::max<size_t>(1, max_txs);
  app->window.max_wait_us = std::max<int64_t>(0, max_wait_us);
}

int gvh_checktx(gvh_app* app, const uint8_t* tx, size_t tx_len, gvh_result* out) {
  if (!app || (!tx && tx_len) || !out) return GVH_EINVAL;
  Window& w = app->window;
  int rc = GVH_OK;
  struct Inflight {
    Window& w;
    ~Inflight() { w.inflight.fetch_sub(1); }
  };
  {
    std::unique_lock<std::mutex> lk(w.m);
    const bool lone = !w.open && w.inflight.load() == 0 && w.last_size.load() <= 1;
    w.inflight.fetch_add(1);
    Inflight guard{w};
    if (lone || w.max_wait_us == 0) {
      // Nothing else can join (tendermint v0.33 delivers CheckTx one call at
      // a time, baseapp/abci.go:165-196): no window, the ante chain verifies
      // this tx's leaves in its own GPU batch right away.
      w.last_size.store(1);
      app->st_windows += 1;
      app->st_window_txs += 1;
      lk.unlock();
      return ante_bytes(app, tx, tx_len, false, out);
    }
    if (!w.open) {
      w.open = std::make_shared<Window::Batch>();
      w.open->deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(w.max_wait_us);
    }
    auto b = w.open;
    b->items.emplace_back(tx, tx_len);
    auto flush = [&]() {                              // this caller verifies the window's batch
      w.open = nullptr;
      b->flushing = true;
      w.last_size.store(b->items.size());
      lk.unlock();
      std::vector<const uint8_t*> ptrs;
      std::vector<size_t> ls;
      for (auto& it : b->items) { ptrs.push_back(it.first); ls.push_back(it.second); }
      const int r = preverify(app, ptrs.size(), ptrs.data(), ls.data(), nullptr, nullptr, true);
      app->st_windows += 1;
      app->st_window_txs += ptrs.size();
      lk.lock();
      b->done = true;
      w.cv.notify_all();
      return r;
    };
    if (b->items.size() >= w.max_txs) rc = flush();
    else
      while (!b->done) {
        if (b->flushing) { w.cv.wait(lk); continue; }
        if (w.cv.wait_until(lk, b->deadline) == std::cv_status::timeout && !b->done && !b->flushing && w.open == b)
          rc = flush();
      }
    lk.unlock();
    if (rc == GVH_EDEVICE) return rc;                // the GPU failed: the caller falls back
    return ante_bytes(app, tx, tx_len, false, out);
  }
}

int gvh_consume_sig_gas(gvh_app* app, const uint8_t* sig, size_t sig_len, const uint8_t* pub_amino, size_t pub_len,
                        uint64_t gas_limit, gvh_result* out) {
  if (!app || !out) return GVH_EINVAL;
  GasMeter gm{gas_limit == 0, gas_limit};
  Span sg{sig, sig ? sig_len : 0};
  try {
    if (!pub_amino || !pub_len) {
      SdkError e = wrap(kErrInvalidPubKey, "unrecognized public key type: <nil>");
      copy_result(out, &e, gm.used, 0, 0, 0);
      return GVH_OK;
    }
    PubKey pk = decode_pubkey(pub_amino, pub_len);
    SdkError e;
    if (!consume_sig_gas(gm, sg, pk, app, &e)) copy_result(out, &e, gm.used, 0, 0, 0);
    else copy_result(out, nullptr, gm.used, 0, 0, 0);
  } catch (const Panic& p) {
    SdkError e = wrap(kErrPanic, p.what());
    copy_result(out, &e, gm.used, 0, 0, 0);
  } catch (const OutOfGas& o) {
    SdkError e = wrap(kErrOutOfGas, std::string("out of gas in location: ") + o.descriptor);
    copy_result(out, &e, gm.used, 0, 0, 0);
  }
  return GVH_OK;
}

void gvh_cache_clear(gvh_app* app) {
  app->cache.clear();
  app->memo.clear();
}
size_t gvh_cache_size(gvh_app* app) { return app->cache.size(); }
void gvh_set_cache_capacity(gvh_app* app, size_t entries) { app->cache.resize(std::max<size_t>(entries, 512)); }

void gvh_set_keyed(gvh_app* app, int keyed, size_t load_min) {
  std::lock_guard<std::mutex> g(app->gpu_mu);
  std::unique_lock<std::shared_mutex> wk(app->key_mu);
  app->keyed = keyed != 0;
  app->key_load_min = load_min;
}

void gvh_set_gpu_hash(gvh_app* app, int on) {
  std::lock_guard<std::mutex> g(app->mu);
  app->gpu_hash = on != 0;
}
int gvh_get_gpu_hash(gvh_app* app) {
  std::lock_guard<std::mutex> g(app->mu);
  return app->gpu_hash ? 1 : 0;
}

void gvh_get_keyed(gvh_app* app, int* keyed, size_t* load_min, size_t* key_cap) {
  std::lock_guard<std::mutex> g(app->gpu_mu);
  if (keyed) *keyed = app->keyed ? 1 : 0;
  if (load_min) *load_min = app->key_load_min;
  if (key_cap) *key_cap = app->key_cap;
}
void gvh_set_threads(gvh_app* app, int threads) {
  if (!app) return;
  std::lock_guard<std::mutex> g(app->pool_mu);
  app->threads = std::max(1, std::min(256, threads));
  app->pool.reset(new Pool(app->threads - 1));
}

void gvh_get_stats(gvh_app* app, gvh_stats* o) {
  memset(o, 0, sizeof *o);
  o->gpu_calls = app->st_gpu_calls;
  o->gpu_leaves = app->st_gpu_leaves;
  o->cache_hits = app->st_hits;
  o->cache_misses = app->st_misses;
  o->memo_hits = app->st_memo;
  o->windows = app->st_windows;
  o->window_txs = app->st_window_txs;
  o->cache_entries = app->cache.size();
  o->cache_capacity = app->cache.capacity();
  o->preverify_ns = app->st_pre_ns;
  o->gpu_ns = app->st_gpu_ns;
  o->deliver_loop_ns = app->st_loop_ns;
}

size_t gvh_std_sign_bytes(const char* chain_id, uint64_t accnum, uint64_t seq, const char* fee_json,
                          const char* const* msgs_json, size_t n_msgs, const char* memo, uint8_t* out, size_t cap) {
  std::string s = "{\"account_number\":\"" + std::to_string(accnum) + "\",\"chain_id\":" +
                  go_json_string(chain_id ? chain_id : "") + ",\"fee\":" + (fee_json ? fee_json : "") + ",\"memo\":" +
                  go_json_string(memo ? memo : "") + ",\"msgs\":[";
  for (size_t i = 0; i < n_msgs; ++i) {
    if (i) s += ",";
    s += msgs_json[i];
  }
  s += "],\"sequence\":\"" + std::to_string(seq) + "\"}";
  if (out) memcpy(out, s.data(), std::min(cap, s.size()));
  return s.size();
}

size_t gvh_tx_sign_bytes(const uint8_t* tx, size_t tx_len, const char* chain_id, uint64_t accnum, uint64_t seq,
                         uint8_t* out, size_t cap, char* err, size_t err_cap) {
  try {
    auto t = decode_tx(tx, tx_len, false);
    const std::string s = sign_bytes(*t, go_json_string(chain_id ? chain_id : ""), accnum, seq);
    if (out) memcpy(out, s.data(), std::min(cap, s.size()));
    if (err && err_cap) err[0] = 0;
    return s.size();
  } catch (const AminoErr& e) {
    if (err && err_cap) snprintf(err, err_cap, "%s", e.what());
    return 0;
  }
}

int gvh_pubkey_address(const uint8_t* pub, size_t len, uint8_t out20[20]) {
  try {
    PubKey pk = decode_pubkey(pub, len);
    auto a = pubkey_address(pk);
    memcpy(out20, a.data(), 20);
    return 0;
  } catch (const Panic&) {
    return GVH_EINVAL;
  }
}

size_t gvh_bech32_address(const uint8_t addr20[20], char* out, size_t cap) {
  std::string s = acc_string(addr20, 20);
  if (out && cap) snprintf(out, cap, "%s", s.c_str());
  return s.size();
}

}  // extern "C"

// ---- IBC 07-tendermint light-client commit checks.
//
// x/ibc/07-tendermint/update.go:88 (lite.Verify -> VerifyAdjacent /
// VerifyNonAdjacent) and misbehaviour.go:88-97 check validator commits with
// tendermint v0.33.4 types/validator_set.go VerifyCommit (signature i <->
// validator i, +2/3 of the total power, every present signature checked) and
// VerifyCommitTrusting (validators found by address, trust level of the
// total power, double votes rejected, returns as soon as the tally passes).
// Each commit's loop stops at its first wrong signature.  Here every
// signature any commit's loop could read -- present, validator known, 64
// bytes long (tendermint's ed25519 VerifyBytes rejects other lengths without
// verifying) -- of every commit in the call is verified in ONE
// gv_verify_ed25519_msgs batch, then each loop is walked in reference order
// over the verdicts.  A signature verified beyond the point where the
// reference would have stopped is never read, so results (code, index,
// tallies) are the sequential loop's.
extern "C" int gvh_verify_commits(gvh_app* app, size_t n, const gvh_commit* commits, gvh_commit_result* out) {
  if (!app || (n && (!commits || !out))) return GVH_EINVAL;
  using AddrKey = std::array<uint8_t, 20>;
  struct AddrHash {
    size_t operator()(const AddrKey& a) const {
      uint64_t v;
      memcpy(&v, a.data(), 8);
      return (size_t)(v * 0x9E3779B97F4A7C15ull);
    }
  };
  std::vector<std::vector<int32_t>> vidx(n);        // per signature: the validator its loop would read (-1: none)
  std::vector<std::vector<int32_t>> item(n);        // per signature: its batch item (-1: false without verifying)
  // two batches: trusted sets (keys loaded into the arena: a validator set
  // signs block after block) and relayer-supplied sets (keys not loaded)
  struct EdB {
    std::vector<uint8_t> pub, sig, blob, ok;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    size_t m = 0;
  } bt[2];
  std::vector<uint8_t> plain(n, 0);                 // per commit: its items are in bt[1]
  for (size_t c = 0; c < n; ++c) {
    const gvh_commit& k = commits[c];
    gvh_commit_result& r = out[c];
    r = gvh_commit_result{GVH_COMMIT_OK, -1, -1, 0, 0};
    if ((k.n_vals && (!k.val_pub32 || !k.val_power || (k.trusting && !k.val_addr20))) ||
        (k.n_sigs && (!k.flag || !k.sig64 || !k.sig_len || !k.msg_off || !k.msg_len || (k.trusting && !k.sig_addr20))))
      return GVH_EINVAL;
    if (k.trusting) {
      // "trustLevel must be within [1/3, 1]": the reference panics
      if (k.trust_den <= 0 || k.trust_num * 3 < k.trust_den || k.trust_num > k.trust_den) {
        r.code = GVH_COMMIT_BAD_TRUST;
        continue;
      }
      if (!k.basic_ok) { r.code = GVH_COMMIT_BASIC; continue; }
    } else {
      if (k.n_vals != k.n_sigs) { r.code = GVH_COMMIT_SIZE; continue; }   // checked before verifyCommitBasic
      if (!k.basic_ok) { r.code = GVH_COMMIT_BASIC; continue; }
    }
    std::unordered_map<AddrKey, int32_t, AddrHash> by_addr;
    if (k.trusting) {
      by_addr.reserve(k.n_vals * 2);
      for (size_t v = 0; v < k.n_vals; ++v) {
        AddrKey a;
        memcpy(a.data(), k.val_addr20 + 20 * v, 20);
        by_addr.emplace(a, (int32_t)v);               // addresses are unique in a validator set
      }
    }
    vidx[c].assign(k.n_sigs, -1);
    item[c].assign(k.n_sigs, -1);
    for (size_t i = 0; i < k.n_sigs; ++i) {
      if (k.flag[i] == GVH_COMMIT_FLAG_ABSENT) continue;
      int32_t v = (int32_t)i;
      if (k.trusting) {
        AddrKey a;
        memcpy(a.data(), k.sig_addr20 + 20 * i, 20);
        auto it = by_addr.find(a);
        v = it == by_addr.end() ? -1 : it->second;
      }
      vidx[c][i] = v;
      if (v < 0 || k.sig_len[i] != 64) continue;
      plain[c] = k.keys_trusted ? 0 : 1;
      EdB& e = bt[plain[c]];
      item[c][i] = (int32_t)e.m++;
      e.pub.insert(e.pub.end(), k.val_pub32 + 32 * (size_t)v, k.val_pub32 + 32 * (size_t)v + 32);
      e.sig.insert(e.sig.end(), k.sig64 + 64 * i, k.sig64 + 64 * i + 64);
      e.off.push_back(e.blob.size());
      e.len.push_back(k.msg_len[i]);
      if (k.msg_len[i])
        e.blob.insert(e.blob.end(), k.msg_blob + k.msg_off[i], k.msg_blob + k.msg_off[i] + k.msg_len[i]);
    }
  }
  for (int t = 0; t < 2; ++t) {
    EdB& e = bt[t];
    e.ok.assign(e.m, 0);
    if (!e.m) continue;
    if (!app->gpu) return GVH_ENOVERIFIER;
    std::lock_guard<std::mutex> g(app->gpu_mu);
    // a trusted validator set signs block after block: its keys are loaded
    // once; a relayer-supplied set is verified without touching the arena
    if (verify_ed(app, e.m, e.pub.data(), e.sig.data(), e.blob.empty() ? nullptr : e.blob.data(), e.off.data(),
                  e.len.data(), e.ok.data(), t == 0) != GV_OK)
      return GVH_EDEVICE;
    app->st_gpu_calls += 1;
    app->st_gpu_leaves += e.m;
  }
  for (size_t c = 0; c < n; ++c) {
    const gvh_commit& k = commits[c];
    gvh_commit_result& r = out[c];
    if (r.code != GVH_COMMIT_OK) continue;
    int64_t total = 0;
    for (size_t v = 0; v < k.n_vals; ++v) total += k.val_power[v];
    const int64_t needed = k.trusting ? total * k.trust_num / k.trust_den : total * 2 / 3;
    int64_t tallied = 0;
    std::unordered_map<int32_t, int32_t> seen;        // trusting: validator -> first commit index
    bool passed = false;
    for (size_t i = 0; i < k.n_sigs && r.code == GVH_COMMIT_OK && !passed; ++i) {
      if (k.flag[i] == GVH_COMMIT_FLAG_ABSENT) continue;
      const int32_t v = vidx[c][i];
      if (k.trusting) {
        if (v < 0) continue;                          // unknown validator: skipped
        auto it = seen.find(v);
        if (it != seen.end()) {
          r.code = GVH_COMMIT_DOUBLE_VOTE;
          r.idx = it->second;
          r.idx2 = (int32_t)i;
          break;
        }
        seen.emplace(v, (int32_t)i);
      }
      const bool good = item[c][i] >= 0 && bt[plain[c]].ok[(size_t)item[c][i]] != 0;
      if (!good) {
        r.code = GVH_COMMIT_WRONG_SIG;
        r.idx = (int32_t)i;
        break;
      }
      if (k.flag[i] == GVH_COMMIT_FLAG_COMMIT) tallied += k.val_power[v];   // blockID.Equals(commitSig.BlockID(...))
      if (k.trusting && tallied > needed) passed = true;
    }
    r.got = tallied;
    r.needed = needed;
    if (r.code == GVH_COMMIT_OK && !passed && tallied <= needed) r.code = GVH_COMMIT_NOT_ENOUGH;
  }
  return GVH_OK;
}
