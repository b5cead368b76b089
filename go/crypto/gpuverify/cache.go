package gpuverify

import (
	"container/list"
	"crypto/sha256"
	"sync"
)

// Leaf kinds in a verdict-cache key.
const (
	KindSecp256k1 byte = 0
	KindEd25519   byte = 1
)

// LeafKey is the verdict-cache key of one VerifyBytes(msg, sig) leaf:
// SHA256(kind || pub || sig || SHA256(msg)).  A secp256k1 verdict depends on
// msg only through SHA256(msg) (tendermint crypto.Sha256 -> ecdsa.Verify), an
// ed25519 verdict on msg itself -- which SHA256(msg) identifies (collision
// resistance) -- so a cached verdict is exactly the reference's answer.
func LeafKey(kind byte, pub, sig, msg []byte) [32]byte {
	h := sha256.Sum256(msg)
	b := make([]byte, 0, 1+len(pub)+len(sig)+32)
	b = append(b, kind)
	b = append(b, pub...)
	b = append(b, sig...)
	b = append(b, h[:]...)
	return sha256.Sum256(b)
}

// VerdictCache is a bounded LRU map LeafKey -> verdict, safe for concurrent
// use.  PreVerifyTxs fills it; BatchSigVerificationDecorator reads it.
type VerdictCache struct {
	mu  sync.Mutex
	cap int
	m   map[[32]byte]*list.Element
	ll  *list.List
}

type cacheEntry struct {
	key [32]byte
	ok  bool
}

// NewVerdictCache returns a cache holding at most capacity verdicts.
func NewVerdictCache(capacity int) *VerdictCache {
	if capacity < 1 {
		capacity = 1
	}
	return &VerdictCache{cap: capacity, m: make(map[[32]byte]*list.Element, capacity), ll: list.New()}
}

// Get returns (verdict, true) on a hit.
func (c *VerdictCache) Get(k [32]byte) (bool, bool) {
	c.mu.Lock()
	defer c.mu.Unlock()
	if e, ok := c.m[k]; ok {
		c.ll.MoveToFront(e)
		return e.Value.(*cacheEntry).ok, true
	}
	return false, false
}

// Put records a verdict, evicting the least recently used entry when full.
func (c *VerdictCache) Put(k [32]byte, ok bool) {
	c.mu.Lock()
	defer c.mu.Unlock()
	if e, hit := c.m[k]; hit {
		e.Value.(*cacheEntry).ok = ok
		c.ll.MoveToFront(e)
		return
	}
	if c.ll.Len() >= c.cap {
		old := c.ll.Back()
		c.ll.Remove(old)
		delete(c.m, old.Value.(*cacheEntry).key)
	}
	c.m[k] = c.ll.PushFront(&cacheEntry{k, ok})
}

// Len is the number of cached verdicts.
func (c *VerdictCache) Len() int {
	c.mu.Lock()
	defer c.mu.Unlock()
	return c.ll.Len()
}
