// gvhost.cpp -- host-side mirror of the reference's signature-verification
// ante path (see gvhost.h for the file:line map), batching every secp256k1
// leaf of a transaction (or of a whole block via gvh_preverify) into one
// libgpuverify call.
#include "gvhost.h"

#include <openssl/evp.h>
#include <openssl/ripemd.h>
#include <openssl/sha.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

using Bytes = std::vector<uint8_t>;

// ------------------------------------------------------------------ errors
// sdkerrors codes (types/errors/errors.go)
constexpr uint32_t kErrTxDecode = 2, kErrUnauthorized = 4, kErrInvalidPubKey = 8, kErrUnknownAddress = 9,
                   kErrOutOfGas = 11, kErrTooManySignatures = 14, kErrPanic = 111222;

struct SdkError {
  uint32_t code;
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
    case kErrTooManySignatures: return "maximum number of signatures exceeded";
    case kErrPanic: return "panic";
    default: return "internal";
  }
}
// sdkerrors.Wrap(err, msg).Error() == msg + ": " + err.Error()
SdkError wrap(uint32_t code, const std::string& msg) {
  return SdkError{code, code == kErrPanic ? "undefined" : "sdk", msg + ": " + err_desc(code)};
}

// Thrown where the reference panics (amino MustUnmarshal, index out of range);
// runTx recovers it into ErrPanic (baseapp/baseapp.go:490-512).
struct Panic : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct OutOfGas {
  std::string descriptor;
};

// ---------------------------------------------------------------- hashing
// The one-shot SHA256() of OpenSSL 3 fetches the digest through the provider
// store on every call (a global lock: no scaling across PreVerifyTxs threads);
// the context API hashes with no shared state.
std::array<uint8_t, 32> sha256(const uint8_t* p, size_t n) {
  std::array<uint8_t, 32> o;
  SHA256_CTX c;
  SHA256_Init(&c);
  SHA256_Update(&c, p, n);
  SHA256_Final(o.data(), &c);
  return o;
}

// ------------------------------------------------------------------ bech32
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
std::string acc_string(const std::array<uint8_t, 20>& a) { return bech32("cosmos", a.data(), 20); }

// --------------------------------------------------- Go encoding/json strings
// json.Marshal(string): escapes '"', '\\', control chars, HTML <>&, U+2028/9;
// invalid UTF-8 becomes U+FFFD.
std::string go_json_string(const std::string& s) {
  std::string o = "\"";
  static const char* hex = "0123456789abcdef";
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = (unsigned char)s[i];
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
    // decode one UTF-8 sequence
    int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    uint32_t cp = 0;
    bool ok = len && i + len <= s.size();
    if (ok) {
      cp = c & (0x7F >> len);
      for (int k = 1; k < len; ++k) {
        unsigned char cc = (unsigned char)s[i + k];
        if ((cc & 0xC0) != 0x80) { ok = false; break; }
        cp = (cp << 6) | (cc & 0x3F);
      }
      if (ok && ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
                 (cp >= 0xD800 && cp <= 0xDFFF)))
        ok = false;
    }
    if (!ok) { o += "\xEF\xBF\xBD"; ++i; continue; }
    if (cp == 0x2028 || cp == 0x2029) { o += cp == 0x2028 ? "\\u2028" : "\\u2029"; }
    else o.append(s, i, len);
    i += len;
  }
  return o + "\"";
}

// ------------------------------------------------------------------- amino
// Registered prefixes (crypto/encode_test.go:51-60, tendermint crypto codec).
const uint8_t kPrefixSecp[4] = {0xEB, 0x5A, 0xE9, 0x87};
const uint8_t kPrefixEd[4] = {0x16, 0x24, 0xDE, 0x64};
const uint8_t kPrefixMulti[4] = {0x22, 0xC1, 0xF7, 0xE2};

struct Reader {
  const uint8_t* p;
  size_t n, i = 0;
  Reader(const uint8_t* p_, size_t n_) : p(p_), n(n_) {}
  bool done() const { return i >= n; }
  uint64_t uvarint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (i >= n) throw Panic("EOF reading uvarint");
      uint8_t b = p[i++];
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    throw Panic("uvarint overflow");
  }
  Bytes bytes() {
    uint64_t len = uvarint();
    if (len > n - i) throw Panic("byte slice length out of range");
    Bytes b(p + i, p + i + len);
    i += len;
    return b;
  }
};

struct PubKey {
  enum Kind { Secp256k1, Ed25519, Multisig } kind;
  std::array<uint8_t, 33> secp{};
  std::array<uint8_t, 32> ed{};
  uint64_t k = 0;
  std::vector<PubKey> subs;
  Bytes amino;   // the exact bytes (multisig address)
};

PubKey decode_pubkey(const uint8_t* p, size_t n, int depth = 0) {
  if (depth > 8) throw Panic("multisig nesting too deep");
  if (n < 4) throw Panic("amino: prefix too short");
  PubKey pk;
  pk.amino.assign(p, p + n);
  Reader r(p + 4, n - 4);
  if (!memcmp(p, kPrefixSecp, 4)) {
    pk.kind = PubKey::Secp256k1;
    Bytes b = r.bytes();
    if (b.size() != 33 || !r.done()) throw Panic("amino: bad secp256k1 pubkey");
    memcpy(pk.secp.data(), b.data(), 33);
  } else if (!memcmp(p, kPrefixEd, 4)) {
    pk.kind = PubKey::Ed25519;
    Bytes b = r.bytes();
    if (b.size() != 32 || !r.done()) throw Panic("amino: bad ed25519 pubkey");
    memcpy(pk.ed.data(), b.data(), 32);
  } else if (!memcmp(p, kPrefixMulti, 4)) {
    pk.kind = PubKey::Multisig;
    int last_field = 0;
    while (!r.done()) {
      uint64_t key = r.uvarint();
      int field = (int)(key >> 3), typ = (int)(key & 7);
      if (field < last_field || (field == last_field && field != 2)) throw Panic("amino: field order");
      last_field = field;
      if (field == 1 && typ == 0) pk.k = r.uvarint();
      else if (field == 2 && typ == 2) {
        Bytes b = r.bytes();
        pk.subs.push_back(decode_pubkey(b.data(), b.size(), depth + 1));
      } else throw Panic("amino: unexpected field in PubKeyMultisigThreshold");
    }
  } else {
    throw Panic("amino: unregistered concrete type prefix");
  }
  return pk;
}

// tendermint libs/bits CompactBitArray
struct CompactBitArray {
  bool present = false;
  uint8_t extra = 0;
  Bytes elems;
  int size() const {
    if (!present) return 0;
    if (extra == 0) return (int)elems.size() * 8;
    return ((int)elems.size() - 1) * 8 + extra;
  }
  bool get(int i) const {
    if (i < 0 || i >= size()) return false;
    return (elems[i >> 3] & (uint8_t)(1u << (7 - (i % 8)))) != 0;
  }
  int true_bits_before(int idx) const {
    int c = 0;
    for (int i = 0; i < idx && i < size(); ++i) c += get(i);
    return c;
  }
};
struct Multisignature {
  CompactBitArray bits;
  std::vector<Bytes> sigs;
};
Multisignature decode_multisig(const Bytes& b) {
  Multisignature m;
  Reader r(b.data(), b.size());
  int last_field = 0;
  while (!r.done()) {
    uint64_t key = r.uvarint();
    int field = (int)(key >> 3), typ = (int)(key & 7);
    if (field < last_field || (field == last_field && field != 2)) throw Panic("amino: field order");
    last_field = field;
    if (field == 1 && typ == 2) {
      Bytes cb = r.bytes();
      Reader rc(cb.data(), cb.size());
      m.bits.present = true;
      int lf = 0;
      while (!rc.done()) {
        uint64_t k2 = rc.uvarint();
        int f2 = (int)(k2 >> 3), t2 = (int)(k2 & 7);
        if (f2 <= lf) throw Panic("amino: field order");
        lf = f2;
        if (f2 == 1 && t2 == 0) {
          uint64_t v = rc.uvarint();
          if (v > 255) throw Panic("amino: byte overflow");
          m.bits.extra = (uint8_t)v;
        } else if (f2 == 2 && t2 == 2) {
          m.bits.elems = rc.bytes();
        } else throw Panic("amino: unexpected field in CompactBitArray");
      }
      if (m.bits.extra >= 8 || (m.bits.extra && m.bits.elems.empty())) throw Panic("amino: invalid CompactBitArray");
    } else if (field == 2 && typ == 2) {
      m.sigs.push_back(r.bytes());
    } else throw Panic("amino: unexpected field in Multisignature");
  }
  return m;
}

int count_subkeys(const PubKey& pk) {  // types.CountSubKeys (stdtx.go:125-137)
  if (pk.kind != PubKey::Multisig) return 1;
  int c = 0;
  for (auto& s : pk.subs) c += count_subkeys(s);
  return c;
}

std::array<uint8_t, 20> pubkey_address(const PubKey& pk) {
  std::array<uint8_t, 20> a{};
  if (pk.kind == PubKey::Secp256k1) {
    auto h = sha256(pk.secp.data(), 33);
    RIPEMD160_CTX c;                                  // context API: no provider fetch per call
    RIPEMD160_Init(&c);
    RIPEMD160_Update(&c, h.data(), 32);
    RIPEMD160_Final(a.data(), &c);
  } else if (pk.kind == PubKey::Ed25519) {
    auto h = sha256(pk.ed.data(), 32);
    memcpy(a.data(), h.data(), 20);
  } else {
    auto h = sha256(pk.amino.data(), pk.amino.size());
    memcpy(a.data(), h.data(), 20);
  }
  return a;
}

bool ed25519_verify(const std::array<uint8_t, 32>& pub, const Bytes& msg, const Bytes& sig) {
  if (sig.size() != 64) return false;
  EVP_PKEY* k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, pub.data(), 32);
  if (!k) return false;
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  bool ok = c && EVP_DigestVerifyInit(c, nullptr, nullptr, nullptr, k) == 1 &&
            EVP_DigestVerify(c, sig.data(), sig.size(), msg.data(), msg.size()) == 1;
  EVP_MD_CTX_free(c);
  EVP_PKEY_free(k);
  return ok;
}

// --------------------------------------------------------------- flat tx
struct FlatTx {
  std::vector<std::string> msgs;
  std::string fee, memo;
  std::vector<std::array<uint8_t, 20>> signers;
  std::vector<Bytes> sig_pubs, sigs;
};
struct FlatReader {
  const uint8_t* p;
  size_t n, i = 0;
  uint32_t u32() {
    if (i + 4 > n) throw std::invalid_argument("truncated tx");
    uint32_t v = p[i] | (p[i + 1] << 8) | (p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24);
    i += 4;
    return v;
  }
  Bytes bytes() {
    uint32_t l = u32();
    if (l > n - i) throw std::invalid_argument("truncated tx");
    Bytes b(p + i, p + i + l);
    i += l;
    return b;
  }
};
FlatTx parse_flat(const uint8_t* p, size_t n) {
  FlatReader r{p, n};
  FlatTx t;
  uint32_t nm = r.u32();
  for (uint32_t k = 0; k < nm; ++k) { Bytes b = r.bytes(); t.msgs.emplace_back(b.begin(), b.end()); }
  { Bytes b = r.bytes(); t.fee.assign(b.begin(), b.end()); }
  { Bytes b = r.bytes(); t.memo.assign(b.begin(), b.end()); }
  uint32_t ns = r.u32();
  for (uint32_t k = 0; k < ns; ++k) {
    if (r.i + 20 > n) throw std::invalid_argument("truncated tx");
    std::array<uint8_t, 20> a;
    memcpy(a.data(), p + r.i, 20);
    r.i += 20;
    t.signers.push_back(a);
  }
  uint32_t nsig = r.u32();
  for (uint32_t k = 0; k < nsig; ++k) {
    t.sig_pubs.push_back(r.bytes());
    t.sigs.push_back(r.bytes());
  }
  if (r.i != n) throw std::invalid_argument("trailing bytes in tx");
  return t;
}

std::string std_sign_bytes(const std::string& chain, uint64_t accnum, uint64_t seq, const std::string& fee,
                           const std::vector<std::string>& msgs, const std::string& memo) {
  // StdSignDoc keys are already in sorted order and every embedded JSON is
  // canonical (MustSortJSON output), so composing canonical pieces equals
  // MustSortJSON(amino.MarshalJSON(StdSignDoc{...})).
  std::string o = "{\"account_number\":\"" + std::to_string(accnum) + "\",\"chain_id\":" + go_json_string(chain) +
                  ",\"fee\":" + fee + ",\"memo\":" + go_json_string(memo) + ",\"msgs\":[";
  for (size_t i = 0; i < msgs.size(); ++i) {
    if (i) o += ",";
    o += msgs[i];
  }
  o += "],\"sequence\":\"" + std::to_string(seq) + "\"}";
  return o;
}

// ----------------------------------------------------------- app / state
// simSecp256k1Pubkey (x/auth/ante/sigverify.go:27-31), amino-encoded
const Bytes kSimSecp256k1Pubkey = {0xEB, 0x5A, 0xE9, 0x87, 0x21, 0x03, 0x5A, 0xD6, 0x81, 0x0A, 0x47, 0xF0, 0x73, 0x55,
                                   0x3F, 0xF3, 0x0D, 0x2F, 0xCC, 0x7E, 0x0D, 0x3B, 0x1C, 0x0B, 0x74, 0xB6, 0x1A, 0x1A,
                                   0xAA, 0x25, 0x82, 0x34, 0x40, 0x37, 0x15, 0x1E, 0x14, 0x3A};

struct Account {
  uint64_t number = 0, sequence = 0;
  Bytes pub;   // amino, empty = not set
};
struct AddrHash {
  size_t operator()(const std::array<uint8_t, 20>& a) const {
    size_t h;
    memcpy(&h, a.data(), sizeof h);
    return h;
  }
};

}  // namespace

struct gvh_app {
  gv_ctx* gpu = nullptr;
  uint64_t sig_limit = 7, cost_secp = 1000, cost_ed = 590;
  std::string chain_id = "";
  int64_t height = 1;
  bool recheck = false;
  uint64_t gas_limit = 0;
  std::unordered_map<std::array<uint8_t, 20>, Account, AddrHash> accounts;
  std::unordered_map<std::string, bool> cache;   // pub33 || sig64 || sha256(msg)
  std::mutex mu;
  // PreVerifyTxs host threads: measured on the MI355X box host (tools/host_probe.py,
  // 10k MsgSend txs) 1 thread 11-12 ms, 4 threads 9.4 ms, 16 threads 11.4 ms --
  // the stages are allocation-heavy and stop scaling past a few threads.
  int threads = std::max(1, std::min(4, (int)std::thread::hardware_concurrency()));
};

namespace {

struct GasMeter {
  uint64_t limit, used = 0;
  void consume(uint64_t amount, const char* desc) {
    used += amount;
    if (limit && used > limit) throw OutOfGas{desc};
  }
};

// One secp256k1 leaf: VerifyBytes(msg, sig) for pub33.
struct Leaf {
  std::array<uint8_t, 33> pub;
  Bytes sig;
  std::array<uint8_t, 32> dig;
  int verdict = -1;    // -1 unknown, 0/1
  std::string key() const {
    std::string k((const char*)pub.data(), 33);
    k.append((const char*)sig.data(), sig.size());
    k.append((const char*)dig.data(), 32);
    return k;
  }
};

// Verification expression for one signer: tendermint VerifyBytes semantics.
struct Node {
  enum Op { Const, SecpLeaf, And } op = Const;
  bool value = false;
  int leaf = -1;
  std::vector<Node> kids;
};

// Build the node for pk.VerifyBytes(msg, sig) (secp256k1_nocgo.go / ed25519 /
// multisig threshold_pubkey.go).  Multisig leaves are AND-ed in bit order; since
// every leaf is a pure function, the AND equals the reference's short-circuit.
Node build_node(const PubKey& pk, const Bytes& msg, const std::array<uint8_t, 32>& dig, const Bytes& sig,
                std::vector<Leaf>& leaves) {
  Node n;
  switch (pk.kind) {
    case PubKey::Secp256k1:
      if (sig.size() != 64) { n.op = Node::Const; n.value = false; return n; }
      n.op = Node::SecpLeaf;
      n.leaf = (int)leaves.size();
      leaves.push_back(Leaf{pk.secp, sig, dig, -1});
      return n;
    case PubKey::Ed25519:
      n.op = Node::Const;
      n.value = ed25519_verify(pk.ed, msg, sig);
      return n;
    case PubKey::Multisig: {
      Multisignature ms;
      try {
        ms = decode_multisig(sig);
      } catch (const Panic&) {
        n.op = Node::Const; n.value = false;     // UnmarshalBinaryBare error -> false
        return n;
      }
      const int size = ms.bits.size();
      if ((int)pk.subs.size() != size || ms.sigs.size() < pk.k || (int)ms.sigs.size() > size ||
          ms.bits.true_bits_before(size) < (int)pk.k) {
        n.op = Node::Const; n.value = false;
        return n;
      }
      n.op = Node::And;
      size_t si = 0;
      for (int i = 0; i < size; ++i) {
        if (!ms.bits.get(i)) continue;
        if (si >= ms.sigs.size()) throw Panic("runtime error: index out of range");
        n.kids.push_back(build_node(pk.subs[i], msg, dig, ms.sigs[si], leaves));
        ++si;
      }
      return n;
    }
  }
  return n;
}

bool eval(const Node& n, const std::vector<Leaf>& leaves) {
  switch (n.op) {
    case Node::Const: return n.value;
    case Node::SecpLeaf: return leaves[n.leaf].verdict == 1;
    case Node::And:
      for (auto& k : n.kids)
        if (!eval(k, leaves)) return false;
      return true;
  }
  return false;
}

// DefaultSigVerificationGasConsumer (sigverify.go:299-322) incl. the multisig
// recursion (ConsumeMultisignatureVerificationGas :325-338, whose nested errors
// are ignored).  Returns an error for the top level only.
bool consume_sig_gas(GasMeter& gm, const Bytes& sig, const PubKey& pk, const gvh_app* app, SdkError* err) {
  switch (pk.kind) {
    case PubKey::Ed25519:
      gm.consume(app->cost_ed, "ante verify: ed25519");
      if (err) *err = wrap(kErrInvalidPubKey, "ED25519 public keys are unsupported");
      return false;
    case PubKey::Secp256k1:
      gm.consume(app->cost_secp, "ante verify: secp256k1");
      return true;
    case PubKey::Multisig: {
      Multisignature ms = decode_multisig(sig);      // MustUnmarshalBinaryBare: panics on error
      const int size = ms.bits.size();
      size_t si = 0;
      for (int i = 0; i < size; ++i) {
        if (!ms.bits.get(i)) continue;
        if (si >= ms.sigs.size() || i >= (int)pk.subs.size()) throw Panic("runtime error: index out of range");
        consume_sig_gas(gm, ms.sigs[si], pk.subs[i], app, nullptr);
        ++si;
      }
      return true;
    }
  }
  return true;
}

void copy_result(gvh_result* out, const SdkError* e, uint64_t gas, uint32_t gpu_leaves, uint32_t hits) {
  memset(out, 0, sizeof *out);
  if (e) {
    out->code = e->code;
    snprintf(out->codespace, sizeof out->codespace, "%s", e->codespace.c_str());
    snprintf(out->log, sizeof out->log, "%s", e->log.c_str());
  }
  out->gas_used = gas;
  out->gpu_leaves = gpu_leaves;
  out->cache_hits = hits;
}

// Resolve every leaf: cache first, misses in ONE gv_verify_digests batch.
int resolve_leaves(gvh_app* app, std::vector<Leaf>& leaves, uint32_t* gpu_leaves, uint32_t* hits) {
  std::vector<size_t> miss;
  for (size_t i = 0; i < leaves.size(); ++i) {
    auto it = app->cache.find(leaves[i].key());
    if (it != app->cache.end()) { leaves[i].verdict = it->second; ++*hits; }
    else miss.push_back(i);
  }
  if (miss.empty()) return GVH_OK;
  if (!app->gpu) return GVH_ENOVERIFIER;
  const size_t m = miss.size();
  std::vector<uint8_t> pub(m * 33), sig(m * 64), dig(m * 32), ok(m);
  for (size_t k = 0; k < m; ++k) {
    const Leaf& L = leaves[miss[k]];
    memcpy(&pub[k * 33], L.pub.data(), 33);
    memcpy(&sig[k * 64], L.sig.data(), 64);
    memcpy(&dig[k * 32], L.dig.data(), 32);
  }
  if (gv_verify_digests(app->gpu, m, pub.data(), sig.data(), dig.data(), ok.data()) != GV_OK) return GVH_EDEVICE;
  for (size_t k = 0; k < m; ++k) {
    leaves[miss[k]].verdict = ok[k];
    app->cache[leaves[miss[k]].key()] = ok[k] != 0;
  }
  *gpu_leaves += (uint32_t)m;
  return GVH_OK;
}

int run_ante(gvh_app* app, const FlatTx& tx, bool simulate, gvh_result* out) {
  GasMeter gm{app->gas_limit};
  uint32_t gpu_leaves = 0, hits = 0;
  auto fail = [&](const SdkError& e) { copy_result(out, &e, gm.used, gpu_leaves, hits); return GVH_OK; };
  try {
    // GetPubKeys(): amino-decode every tx-supplied pubkey (MustUnmarshal -> panic)
    std::vector<std::unique_ptr<PubKey>> tx_pks(tx.sig_pubs.size());
    for (size_t i = 0; i < tx.sig_pubs.size(); ++i)
      if (!tx.sig_pubs[i].empty()) tx_pks[i].reset(new PubKey(decode_pubkey(tx.sig_pubs[i].data(), tx.sig_pubs[i].size())));

    // ---- SetPubKeyDecorator (sigverify.go:60-99)
    for (size_t i = 0; i < tx_pks.size(); ++i) {
      const Bytes* pkb = tx_pks[i] ? &tx.sig_pubs[i] : nullptr;
      if (!pkb) {
        if (!simulate) continue;           // pubkey already set on the account
        pkb = &kSimSecp256k1Pubkey;        // simSecp256k1Pubkey (sigverify.go:19-31)
      }
      if (i >= tx.signers.size()) throw Panic("runtime error: index out of range");
      if (!simulate && pubkey_address(*tx_pks[i]) != tx.signers[i])
        return fail(wrap(kErrInvalidPubKey, "pubKey does not match signer address " + acc_string(tx.signers[i]) +
                                                " with signer index: " + std::to_string(i)));
      auto it = app->accounts.find(tx.signers[i]);
      if (it == app->accounts.end())
        return fail(wrap(kErrUnknownAddress, "account " + acc_string(tx.signers[i]) + " does not exist"));
      if (it->second.pub.empty()) it->second.pub = *pkb;
    }
    // ---- ValidateSigCountDecorator (sigverify.go:275-294)
    {
      uint64_t count = 0;
      for (auto& pk : tx_pks) {
        count += pk ? (uint64_t)count_subkeys(*pk) : 1;   // CountSubKeys(nil) -> 1
        if (count > app->sig_limit)
          return fail(wrap(kErrTooManySignatures,
                           "signatures: " + std::to_string(count) + ", limit: " + std::to_string(app->sig_limit)));
      }
    }
    // ---- SigGasConsumeDecorator (sigverify.go:117-153)
    for (size_t i = 0; i < tx.sigs.size(); ++i) {
      if (i >= tx.signers.size()) throw Panic("runtime error: index out of range");
      auto it = app->accounts.find(tx.signers[i]);
      if (it == app->accounts.end())
        return fail(wrap(kErrUnknownAddress, "account " + acc_string(tx.signers[i]) + " does not exist"));
      PubKey pk;
      if (it->second.pub.empty()) {
        if (!simulate) {
          // a nil pubkey reaches the gas consumer's type switch: "unrecognized public key type: <nil>"
          return fail(wrap(kErrInvalidPubKey, "unrecognized public key type: <nil>"));
        }
        pk.kind = PubKey::Secp256k1;   // simSecp256k1Pubkey
      } else {
        pk = decode_pubkey(it->second.pub.data(), it->second.pub.size());
      }
      SdkError e;
      if (!consume_sig_gas(gm, tx.sigs[i], pk, app, &e)) return fail(e);
    }
    // ---- BatchSigVerificationDecorator (replaces sigverify.go:170-216)
    if (!app->recheck) {
      if (tx.sigs.size() != tx.signers.size())
        return fail(wrap(kErrUnauthorized, "invalid number of signer;  expected: " + std::to_string(tx.signers.size()) +
                                               ", got " + std::to_string(tx.sigs.size())));
      std::vector<Leaf> leaves;
      std::vector<Node> nodes;
      SdkError first_err;
      bool have_err = false;
      for (size_t i = 0; i < tx.sigs.size(); ++i) {
        auto it = app->accounts.find(tx.signers[i]);
        if (it == app->accounts.end()) {
          first_err = wrap(kErrUnknownAddress, "account " + acc_string(tx.signers[i]) + " does not exist");
          have_err = true;
          break;
        }
        const Account& acc = it->second;
        std::string sb = std_sign_bytes(app->chain_id, app->height == 0 ? 0 : acc.number, acc.sequence, tx.fee,
                                        tx.msgs, tx.memo);
        if (!simulate && acc.pub.empty()) {
          first_err = wrap(kErrInvalidPubKey, "pubkey on account is not set");
          have_err = true;
          break;
        }
        if (simulate) continue;
        PubKey pk = decode_pubkey(acc.pub.data(), acc.pub.size());
        Bytes msg(sb.begin(), sb.end());
        auto dig = sha256(msg.data(), msg.size());
        nodes.push_back(build_node(pk, msg, dig, tx.sigs[i], leaves));
      }
      if (!leaves.empty()) {
        int rc = resolve_leaves(app, leaves, &gpu_leaves, &hits);
        if (rc != GVH_OK) return rc;
      }
      for (auto& n : nodes)   // report the FIRST failing signer, as the reference loop does
        if (!eval(n, leaves))
          return fail(wrap(kErrUnauthorized, "signature verification failed; verify correct account sequence and chain-id"));
      if (have_err) return fail(first_err);
    }
    // ---- IncrementSequenceDecorator (sigverify.go:237-259)
    if (!app->recheck || simulate) {
      for (auto& a : tx.signers) {
        auto it = app->accounts.find(a);
        if (it == app->accounts.end()) throw Panic("account not found");
        it->second.sequence += 1;
      }
    }
  } catch (const Panic& p) {
    return fail(wrap(kErrPanic, p.what()));
  } catch (const OutOfGas& o) {
    return fail(wrap(kErrOutOfGas, std::string("out of gas in location: ") + o.descriptor + "; gasWanted: " +
                                       std::to_string(app->gas_limit) + ", gasUsed: " + std::to_string(gm.used)));
  }
  copy_result(out, nullptr, gm.used, gpu_leaves, hits);
  return GVH_OK;
}

// Run fn(i) for i in [0, n) on up to `threads` threads (dynamic chunks).
template <class F>
void parallel_for(size_t n, int threads, F fn) {
  const size_t chunk = 64;
  if (threads <= 1 || n <= chunk) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t lo; (lo = next.fetch_add(chunk)) < n;)
      for (size_t i = lo; i < std::min(n, lo + chunk); ++i) fn(i);
  };
  const int nt = (int)std::min<size_t>(threads, (n + chunk - 1) / chunk);
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
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
  app->sig_limit = lim;
  app->cost_secp = cs;
  app->cost_ed = ce;
}
void gvh_set_context(gvh_app* app, const char* chain_id, int64_t height, int recheck, uint64_t gas_limit) {
  app->chain_id = chain_id ? chain_id : "";
  app->height = height;
  app->recheck = recheck != 0;
  app->gas_limit = gas_limit;
}

int gvh_set_account(gvh_app* app, const uint8_t addr20[20], uint64_t num, uint64_t seq, const uint8_t* pub,
                    size_t pub_len) {
  if (!app || !addr20) return GVH_EINVAL;
  std::array<uint8_t, 20> a;
  memcpy(a.data(), addr20, 20);
  Account acc;
  acc.number = num;
  acc.sequence = seq;
  if (pub && pub_len) acc.pub.assign(pub, pub + pub_len);
  std::lock_guard<std::mutex> lk(app->mu);
  app->accounts[a] = acc;
  return GVH_OK;
}
int gvh_get_account(gvh_app* app, const uint8_t addr20[20], uint64_t* num, uint64_t* seq, uint8_t* pub_out,
                    size_t* pub_len) {
  std::array<uint8_t, 20> a;
  memcpy(a.data(), addr20, 20);
  std::lock_guard<std::mutex> lk(app->mu);
  auto it = app->accounts.find(a);
  if (it == app->accounts.end()) return 0;
  if (num) *num = it->second.number;
  if (seq) *seq = it->second.sequence;
  if (pub_len) *pub_len = it->second.pub.size();
  if (pub_out && !it->second.pub.empty()) memcpy(pub_out, it->second.pub.data(), std::min<size_t>(512, it->second.pub.size()));
  return 1;
}

int gvh_ante(gvh_app* app, const uint8_t* tx, size_t tx_len, int simulate, gvh_result* out) {
  if (!app || !tx || !out) return GVH_EINVAL;
  FlatTx t;
  try {
    t = parse_flat(tx, tx_len);
  } catch (const std::exception&) {
    return GVH_EINVAL;
  }
  std::lock_guard<std::mutex> lk(app->mu);
  return run_ante(app, t, simulate != 0, out);
}

// PreVerifyTxs: (1) decode every tx in parallel, (2) predict each signer's
// sequence in block order (serial: it is a prefix count per signer), (3) build
// sign bytes, SHA-256 and the leaves of every (tx, signer) in parallel (the
// host sign-bytes pipeline of SURVEY.md §8f-3), (4) one GPU batch for the
// cache misses.
int gvh_preverify(gvh_app* app, size_t ntx, const uint8_t* const* txs, const size_t* lens, size_t* n_leaves) {
  if (!app || (ntx && (!txs || !lens))) return GVH_EINVAL;
  std::lock_guard<std::mutex> lk(app->mu);
  auto T0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) { if (getenv("GVH_PROFILE")) { auto t = std::chrono::steady_clock::now(); fprintf(stderr, "%s %.3f ms\n", what, std::chrono::duration<double, std::milli>(t - T0).count()); T0 = t; } };
  std::vector<FlatTx> parsed(ntx);
  std::vector<uint8_t> good(ntx, 0);
  parallel_for(ntx, app->threads, [&](size_t t) {
    try {
      parsed[t] = parse_flat(txs[t], lens[t]);
      good[t] = 1;
    } catch (const std::exception&) {
    }
  });
  lap("parse");
  struct Job {
    const FlatTx* tx;
    size_t signer;
    const Bytes* pub;     // account pubkey, else the tx-supplied one (stable: accounts not modified here)
    uint64_t accnum, seq;
  };
  std::vector<Job> jobs;
  std::unordered_map<std::array<uint8_t, 20>, uint64_t, AddrHash> seq_bump;   // sequence prediction
  seq_bump.reserve(ntx * 2);
  jobs.reserve(ntx);
  for (size_t t = 0; t < ntx; ++t) {
    if (!good[t]) continue;
    const FlatTx& tx = parsed[t];
    for (size_t i = 0; i < tx.sigs.size() && i < tx.signers.size(); ++i) {
      auto it = app->accounts.find(tx.signers[i]);
      if (it == app->accounts.end()) continue;
      const Account& acc = it->second;
      const Bytes* pubb = !acc.pub.empty() ? &acc.pub : (i < tx.sig_pubs.size() ? &tx.sig_pubs[i] : nullptr);
      if (!pubb || pubb->empty()) continue;
      jobs.push_back(Job{&tx, i, pubb, app->height == 0 ? 0 : acc.number, acc.sequence + seq_bump[tx.signers[i]]});
    }
    for (auto& a : tx.signers) seq_bump[a] += 1;
  }
  lap("jobs");
  std::vector<std::vector<Leaf>> job_leaves(jobs.size());
  parallel_for(jobs.size(), app->threads, [&](size_t j) {
    const Job& jb = jobs[j];
    try {
      PubKey pk = decode_pubkey(jb.pub->data(), jb.pub->size());
      std::string sb = std_sign_bytes(app->chain_id, jb.accnum, jb.seq, jb.tx->fee, jb.tx->msgs, jb.tx->memo);
      Bytes msg(sb.begin(), sb.end());
      auto dig = sha256(msg.data(), msg.size());
      build_node(pk, msg, dig, jb.tx->sigs[jb.signer], job_leaves[j]);
    } catch (const Panic&) {
      job_leaves[j].clear();   // malformed: the ante chain will report it; nothing to cache
    }
  });
  lap("signbytes");
  std::vector<Leaf> leaves;
  for (auto& v : job_leaves) leaves.insert(leaves.end(), v.begin(), v.end());
  lap("concat");
  uint32_t gpu_leaves = 0, hits = 0;
  int rc = leaves.empty() ? GVH_OK : resolve_leaves(app, leaves, &gpu_leaves, &hits);
  lap("resolve");
  if (n_leaves) *n_leaves = gpu_leaves;
  return rc;
}

void gvh_set_threads(gvh_app* app, int threads) {
  if (app) app->threads = std::max(1, std::min(256, threads));
}

int gvh_consume_sig_gas(gvh_app* app, const uint8_t* sig, size_t sig_len, const uint8_t* pub_amino, size_t pub_len,
                        uint64_t gas_limit, gvh_result* out) {
  if (!app || !out) return GVH_EINVAL;
  GasMeter gm{gas_limit};
  Bytes sg(sig, sig + (sig ? sig_len : 0));
  try {
    if (!pub_amino || !pub_len) {
      SdkError e = wrap(kErrInvalidPubKey, "unrecognized public key type: <nil>");
      copy_result(out, &e, gm.used, 0, 0);
      return GVH_OK;
    }
    PubKey pk = decode_pubkey(pub_amino, pub_len);
    SdkError e;
    if (!consume_sig_gas(gm, sg, pk, app, &e)) copy_result(out, &e, gm.used, 0, 0);
    else copy_result(out, nullptr, gm.used, 0, 0);
  } catch (const Panic& p) {
    SdkError e = wrap(kErrPanic, p.what());
    copy_result(out, &e, gm.used, 0, 0);
  } catch (const OutOfGas& o) {
    SdkError e = wrap(kErrOutOfGas, std::string("out of gas in location: ") + o.descriptor);
    copy_result(out, &e, gm.used, 0, 0);
  }
  return GVH_OK;
}

void gvh_cache_clear(gvh_app* app) {
  std::lock_guard<std::mutex> lk(app->mu);
  app->cache.clear();
}
size_t gvh_cache_size(gvh_app* app) {
  std::lock_guard<std::mutex> lk(app->mu);
  return app->cache.size();
}

size_t gvh_std_sign_bytes(const char* chain_id, uint64_t accnum, uint64_t seq, const char* fee_json,
                          const char* const* msgs_json, size_t n_msgs, const char* memo, uint8_t* out, size_t cap) {
  std::vector<std::string> msgs;
  for (size_t i = 0; i < n_msgs; ++i) msgs.emplace_back(msgs_json[i]);
  std::string s = std_sign_bytes(chain_id ? chain_id : "", accnum, seq, fee_json ? fee_json : "", msgs, memo ? memo : "");
  if (out) memcpy(out, s.data(), std::min(cap, s.size()));
  return s.size();
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
  std::array<uint8_t, 20> a;
  memcpy(a.data(), addr20, 20);
  std::string s = acc_string(a);
  if (out && cap) snprintf(out, cap, "%s", s.c_str());
  return s.size();
}

}  // extern "C"
