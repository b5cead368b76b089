"""The Go drop-in (go/, source-only: no Go toolchain in this image) against
the tested C++ mirror: the routing policy comes from one place (gpuverify.h
macros read by both), and the decorator's structure keeps the reference's
gas order (the C++ mirror's gas is checked numerically in test_gas_order.py).
"""
import os
import re

import gvhost

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read(*p):
    return open(os.path.join(REPO, *p)).read()


def header_macros():
    h = read("include", "gpuverify.h")
    out = {}
    for name in ("GV_CPU_CROSSOVER", "GV_KEY_LOAD_MIN", "GV_KEY_CAP", "GV_ED_KEY_CAP"):
        m = re.search(r"#define %s \(?(\d+)u?(?: << (\d+))?\)?" % name, h)
        assert m, name
        out[name] = int(m.group(1)) << int(m.group(2) or 0)
    return out


def strip_comments(go: str) -> str:
    return re.sub(r"//[^\n]*", "", go)


def test_policy_constants_shared_by_go_and_cpp():
    mac = header_macros()
    assert mac == {"GV_CPU_CROSSOVER": 4, "GV_KEY_LOAD_MIN": 4096, "GV_KEY_CAP": 1 << 22, "GV_ED_KEY_CAP": 1 << 16}
    app = gvhost.HostApp(None)
    assert app.keyed_policy() == (True, mac["GV_KEY_LOAD_MIN"], mac["GV_KEY_CAP"])
    app.close()
    go = strip_comments(read("go", "crypto", "gpuverify", "gpuverify.go"))
    assert re.search(r"DefaultCPUBelow\s*=\s*int\(C\.GV_CPU_CROSSOVER\)", go)
    assert re.search(r"DefaultKeyLoadMin\s*=\s*int\(C\.GV_KEY_LOAD_MIN\)", go)
    assert re.search(r"DefaultKeyCap\s*=\s*int\(C\.GV_KEY_CAP\)", go)
    assert re.search(r"DefaultEdKeyCap\s*=\s*int\(C\.GV_ED_KEY_CAP\)", go)
    opener = go[go.index("func Open("):go.index("func (g *GPU) Close()")]
    for field in ("CPUBelow: DefaultCPUBelow", "Keyed: true", "KeyLoadMin: DefaultKeyLoadMin",
                  'KeyCap: envInt("GV_KEY_CAP", DefaultKeyCap)', 'EdKeyCap: envInt("GV_ED_KEY_CAP", DefaultEdKeyCap)'):
        assert field in opener, field


def test_go_verify_batch_routes_like_the_mirror():
    go = strip_comments(read("go", "crypto", "gpuverify", "gpuverify.go"))
    vb = go[go.index("func (g *GPU) VerifyBatch("):go.index("func (g *GPU) VerifyBatchPub33(")]
    # CPU below the crossover, then keyed, else pub33 -- in that order
    assert vb.index("g.CPUBelow") < vb.index("g.Keyed") < vb.index("VerifyBatchPub33")
    keyed = go[go.index("func (g *GPU) VerifyBatchKeyed("):]
    # loads only from KeyLoadMin leaves; the lock spans lookup and keyed verify
    assert "g.slotsLocked(pubs, n >= g.KeyLoadMin)" in keyed
    lock, unlock = keyed.index("g.mu.Lock()"), keyed.index("g.mu.Unlock()")
    assert lock < keyed.index("slotsLocked") < keyed.index("gv_verify_msgs_keyed") < unlock
    assert "maxBatchBytes" in keyed                      # oversize split


def test_go_decorator_charges_reads_in_reference_order():
    go = strip_comments(read("go", "x", "auth", "ante", "batch_sigverify.go"))
    ah = go[go.index("func (d BatchSigVerificationDecorator) AnteHandle("):go.index("func (d BatchSigVerificationDecorator) gather(")]
    # look-ahead on a context with its own meter, then the reference loop on ctx
    assert "d.gather(ctx.WithGasMeter(sdk.NewInfiniteGasMeter())" in ah
    loop = ah[ah.index("for i, sig := range sigs"):]
    assert loop.index("GetSignerAcc(ctx, d.ak, signerAddrs[i])") < loop.index("exprs[i].eval(&b)")
    # sign bytes right after the account read, before the nil-key check and the
    # simulate bypass (sigverify.go:201-207)
    assert loop.index("GetSignerAcc(ctx") < loop.index("sigTx.GetSignBytes(ctx, acc)") < \
        loop.index("pubKey == nil") < loop.index("if simulate {")
    assert "return ctx, sdkerrors.Wrap(sdkerrors.ErrUnauthorized" in loop
    gather = go[go.index("func (d BatchSigVerificationDecorator) gather("):go.index("func signBytesNoPanic(")]
    assert "d.ak.GetAccount(look," in gather and "GetSignerAcc(ctx" not in gather
    # unknown / nil sub-keys are deferred to eval (no panic while gathering)
    build = go[go.index("func (b *batch) build("):go.index("func (b *batch) resolve(")]
    assert "cpu: true" in build and "VerifyBytes" not in build.split("default:")[1]
    # the pre-verifier's workers never read the store or a gas meter
    pv = go[go.index("func NewPreVerifier("):]
    assert "ctx.WithGasMeter(sdk.NewInfiniteGasMeter())" in pv
    workers = pv[pv.index("return func() {"):]
    assert "GetAccount" not in workers and "GasMeter" not in workers


def test_go_checktx_window_is_adaptive_and_ingress_releases_lock():
    go = strip_comments(read("go", "baseapp", "preverify.go"))
    join = go[go.index("func (w *CheckTxWindow) join("):go.index("func (w *CheckTxWindow) flush(")]
    assert "lone := w.cur == nil && w.inflight == 0 && w.lastSize <= 1" in join
    assert "full := lone ||" in join
    loop = go[go.index("func (in *Ingress) loop()"):go.index("func (in *Ingress) CheckTx(")]
    # state stage under the lock, GPU stage after it is released
    assert loop.index("in.stateMu.Lock()") < loop.index("prepareCheckTxs(batch)") < \
        loop.index("in.stateMu.Unlock()") < loop.index("verify()")


def test_go_ed25519_routes_like_the_mirror():
    """ed25519 leaves: the Go shim and the C++ mirror (verify_ed) both go keyed
    when every key is resident or the batch has KeyLoadMin leaves, and the
    light-client commit path (Go EdKeyCache, C++ gvh_verify_commits) always
    loads its validator set's keys; the arena is reset at GV_ED_KEY_CAP."""
    go = strip_comments(read("go", "crypto", "gpuverify", "gpuverify.go"))
    vb = go[go.index("func (g *GPU) VerifyBatchEd25519("):go.index("func (g *GPU) VerifyBatchEd25519Cached(")]
    assert "g.verifyEdKeyed(pubs, msgs, sigs, len(pubs) >= g.KeyLoadMin)" in vb
    cached = go[go.index("func (g *GPU) VerifyBatchEd25519Cached("):go.index("func (g *GPU) VerifyBatchEd25519Pub(")]
    assert "g.verifyEdKeyed(pubs, msgs, sigs, true)" in cached
    ek = go[go.index("func (g *GPU) verifyEdKeyed("):]
    lock, unlock = ek.index("g.mu.Lock()"), ek.rindex("g.mu.Unlock()")
    assert lock < ek.index("edSlotsLocked") < ek.index("gv_verify_ed25519_msgs_keyed") < unlock
    assert "g.EdKeyCap" in go[go.index("func (g *GPU) edSlotsLocked("):]
    ibc = strip_comments(read("go", "x", "ibc", "07-tendermint", "batch_verify.go"))
    # only trusted validator sets go through the resident-key path
    assert "ev.(gv.EdKeyCache)" in ibc and "VerifyBatchEd25519Cached(cached.pubs, cached.msgs, cached.sigs)" in ibc
    assert "plain.ok = ev.VerifyBatchEd25519(plain.pubs, plain.msgs, plain.sigs)" in ibc
    assert "if k.KeysTrusted {" in ibc and ibc.count("KeysTrusted: true") == 3 and "full.KeysTrusted = true" in ibc
    cpp = read("cosmos-sdk-rootchain_amd", "host", "gvhost.cpp")
    assert "GV_ED_KEY_CAP" in cpp[cpp.index("int verify_ed("):]
    assert "me >= app->key_load_min" in cpp
    commits = cpp[cpp.index('extern "C" int gvh_verify_commits('):]
    assert re.search(r"verify_ed\(app, e\.m,[^;]*t == 0\)", commits) and "k.keys_trusted ? 0 : 1" in commits


def _split_args(text, start):
    """The top-level arguments of the call whose '(' is at text[start]."""
    depth, args, cur, i = 0, [], "", start
    while i < len(text):
        ch = text[i]
        if ch in "([{":
            depth += 1
            if depth > 1:
                cur += ch
        elif ch in ")]}":
            depth -= 1
            if depth == 0:
                if cur.strip():
                    args.append(cur.strip())
                return args
            cur += ch
        elif ch == "," and depth == 1:
            args.append(cur.strip())
            cur = ""
        else:
            cur += ch
        i += 1
    raise AssertionError("unbalanced call")


def test_go_cgo_calls_match_header_arity():
    """No Go toolchain here: every C.gv_* call in the Go drop-in passes as many
    arguments as include/gpuverify.h declares (the asynchronous gv_submit_* /
    gv_wait calls of SubmitBatch included)."""
    import re
    hdr = open(os.path.join(REPO, "include", "gpuverify.h")).read()
    protos = {}
    for m in re.finditer(r"^[\w\s\*]*?\b(gv_\w+)\(([^;]*?)\);", hdr, re.M | re.S):
        params = [p for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
        if params == ["void"]:
            params = []
        protos[m.group(1)] = len(params)
    assert {"gv_submit_msgs", "gv_submit_msgs_keyed", "gv_wait"} <= set(protos)
    seen = set()
    for root, _, files in os.walk(os.path.join(REPO, "go")):
        for f in files:
            if not f.endswith(".go"):
                continue
            src = open(os.path.join(root, f)).read()
            for m in re.finditer(r"C\.(gv_\w+)\(", src):
                name = m.group(1)
                assert name in protos, name
                args = _split_args(src, m.end() - 1)
                assert len(args) == protos[name], (f, name, len(args), protos[name])
                seen.add(name)
    assert {"gv_submit_msgs", "gv_submit_msgs_keyed", "gv_wait"} <= seen
