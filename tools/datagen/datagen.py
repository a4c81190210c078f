"""Synthetic signature workloads in the libcordagpu C-ABI layout.

Config shapes from SURVEY.md §8(d): N distinct keys (SHA-512("cg-key"||LE64(i))),
xoshiro256** messages, OpenSSL-signed (libcg_datagen.so), and an optional
adversarial fraction split uniformly over the Ed25519 classes E1–E12 — byte
mutations (E1–E6, E12) applied in place, the curve-structured classes (E7–E11)
drawn from the committed golden fixtures (tests/golden/ed25519_golden.json).
"""
from __future__ import annotations

import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "libcg_datagen.so")
L = 2**252 + 27742317777372353535851937790883648493


def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.check_call(["make", "-C", HERE], stdout=subprocess.DEVNULL)
    c = ctypes.CDLL(LIB)
    c.dg_sign_batch.restype = ctypes.c_int
    c.dg_sign_batch.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_int]
    c.dg_fill_bytes.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    c.dg_set_key_options.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    c.dg_txid_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p]
    return c


class Workload:
    """Element-major arrays ready for cg_batch_create / cg_verify_batch."""

    def __init__(self, n, scheme, pk, pk_stride, sig, sig_stride, sig_len, msg, msg_off, msg_len, classes=None):
        self.n, self.scheme, self.pk, self.pk_stride = n, scheme, pk, pk_stride
        self.sig, self.sig_stride, self.sig_len = sig, sig_stride, sig_len
        self.msg, self.msg_off, self.msg_len = msg, msg_off, msg_len
        self.classes = classes

    def tiled(self, n: int) -> "Workload":
        """The first n elements of this workload repeated end to end (a bounded
        pool of distinct signed tuples stretched to a benchmark size).  Every
        copy owns its message bytes, so later in-place mutations stay local."""
        reps = -(-n // self.n)
        m_end = int(self.msg_off[-1]) + int(self.msg_len[-1]) if self.n else 0
        arena = np.concatenate([np.tile(self.msg[:m_end], reps)[:m_end * reps], np.zeros(16, np.uint8)])
        off = (self.msg_off[None, :].astype(np.uint64) + np.arange(reps, dtype=np.uint64)[:, None] * np.uint64(m_end))
        cls = None if self.classes is None else (list(self.classes) * reps)[:n]
        return Workload(n, np.tile(self.scheme, reps)[:n], np.tile(self.pk, (reps, 1))[:n], self.pk_stride,
                        np.tile(self.sig, (reps, 1))[:n], self.sig_stride, np.tile(self.sig_len, reps)[:n], arena,
                        off.ravel()[:n].copy(), np.tile(self.msg_len, reps)[:n], cls)

    def subset(self, idx):
        """Copy of elements idx (messages re-packed)."""
        idx = np.asarray(idx, dtype=np.int64)
        ml = self.msg_len[idx]
        off = np.zeros(len(idx), dtype=np.uint64)
        if len(idx) > 1:
            off[1:] = np.cumsum(ml[:-1], dtype=np.uint64)
        arena = np.concatenate([self.msg[int(self.msg_off[i]):int(self.msg_off[i]) + int(self.msg_len[i])]
                                for i in idx] + [np.zeros(1, np.uint8)])
        return Workload(len(idx), self.scheme[idx].copy(), self.pk[idx].copy(), self.pk_stride, self.sig[idx].copy(),
                        self.sig_stride, self.sig_len[idx].copy(), arena, off, ml.copy(),
                        None if self.classes is None else [self.classes[i] for i in idx])


def make_batch(n: int, msg_bytes: int = 1024, scheme: int | np.ndarray = 4, seed: int = 42, key_base: int = 0,
               threads: int | None = None, sig_stride: int = 72, key_reuse: int = 0,
               ref_seed_stride: int = 0) -> Workload:
    """n signed messages of msg_bytes each (fixed size), all valid.  key_reuse > 0:
    element i signs with key (i mod key_reuse); ref_seed_stride > 0: every such
    element uses the reference's test keys entropyToKeyPair(20..110)."""
    c = lib()
    c.dg_set_key_options(key_reuse, ref_seed_stride)
    threads = threads or min(16, os.cpu_count() or 1)
    sch = np.full(n, scheme, dtype=np.uint8) if np.isscalar(scheme) else np.asarray(scheme, dtype=np.uint8)
    msg = np.empty(n * msg_bytes + 1, dtype=np.uint8)
    c.dg_fill_bytes(msg.ctypes.data, n * msg_bytes, seed)
    msg_off = (np.arange(n, dtype=np.uint64) * msg_bytes)
    msg_len = np.full(n, msg_bytes, dtype=np.uint32)
    pk = np.zeros((n, 64), dtype=np.uint8)
    sig = np.zeros((n, sig_stride), dtype=np.uint8)
    sig_len = np.zeros(n, dtype=np.uint32)
    rc = c.dg_sign_batch(n, sch.ctypes.data, key_base, pk.ctypes.data, 64, sig.ctypes.data, sig_stride,
                         sig_len.ctypes.data, msg.ctypes.data, msg_off.ctypes.data, msg_len.ctypes.data, threads)
    c.dg_set_key_options(0, 0)
    if rc != 0:
        raise RuntimeError("signature generation failed")
    return Workload(n, sch, pk, 64, sig, sig_stride, sig_len, msg, msg_off, msg_len, ["valid"] * n)


ED_CLASSES = ["E1", "E2", "E3", "E4", "E5", "E6", "E7", "E8", "E9", "E10", "E11", "E12"]


def _golden_pool():
    with open(os.path.join(ROOT, "tests", "golden", "ed25519_golden.json")) as f:
        g = json.load(f)
    pool = {}
    for e in g:
        for cls in ("E7", "E8", "E9", "E10", "E11"):
            if e["cls"].startswith(cls + "_"):
                pool.setdefault(cls, []).append(e)
    return pool


def add_ed25519_adversarial(w: Workload, frac: float = 0.01, seed: int = 7) -> Workload:
    """Mutates a fraction of an Ed25519 workload in place, uniformly over E1–E12.
    Structured classes replace the element's key/sig/message with a golden case
    (its message is written over the element's slot, so msg_len may shrink)."""
    rng = np.random.default_rng(seed)
    k = int(round(w.n * frac))
    idx = rng.choice(w.n, size=k, replace=False)
    pool = _golden_pool()
    classes = list(w.classes) if w.classes is not None else ["valid"] * w.n
    for j, i in enumerate(idx):
        cls = ED_CLASSES[j % len(ED_CLASSES)]
        classes[i] = cls
        o, ln = int(w.msg_off[i]), int(w.msg_len[i])
        if cls == "E1":
            w.sig[i, rng.integers(32)] ^= np.uint8(1 << rng.integers(8))
        elif cls == "E2":
            w.sig[i, 32 + rng.integers(32)] ^= np.uint8(1 << rng.integers(8))
        elif cls == "E3":
            if ln:
                w.msg[o + rng.integers(ln)] ^= np.uint8(1 << rng.integers(8))
        elif cls == "E4":
            w.pk[i, :32] = w.pk[(i + 1) % w.n, :32]
        elif cls in ("E5", "E6"):
            s = int.from_bytes(w.sig[i, 32:64].tobytes(), "little")
            t = s + L
            if cls == "E6":
                t = s + 8 * L if s + 8 * L < 2**256 else (2**256 - 1) ^ int(rng.integers(1 << 16))
            if t < 2**256:
                w.sig[i, 32:64] = np.frombuffer(t.to_bytes(32, "little"), dtype=np.uint8)
        elif cls == "E12":
            w.sig_len[i] = int(rng.choice([0, 63, 65]))
        else:
            e = pool[cls][j % len(pool[cls])]
            pk = bytes.fromhex(e["pk"]); sg = bytes.fromhex(e["sig"]); m = bytes.fromhex(e["msg"])
            w.pk[i, :] = 0
            w.pk[i, :32] = np.frombuffer(pk, dtype=np.uint8)
            w.sig[i, :] = 0
            w.sig[i, :len(sg)] = np.frombuffer(sg, dtype=np.uint8)
            w.sig_len[i] = len(sg)
            m = m[:ln]
            w.msg[o:o + len(m)] = np.frombuffer(m, dtype=np.uint8)
            w.msg_len[i] = len(m)
    w.classes = classes
    return w


# ---------------------------------------------------------------- ECDSA (D1–D8)
_N = {2: 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141,
      3: 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551}
EC_CLASSES = ["D1", "D2", "D3", "D4", "D5", "D6", "D7", "D8"]


def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    raw = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(raw)]) + raw


def _der_int(v: int) -> bytes:
    nb = (v.bit_length() + 8) // 8 if v >= 0 else ((v + 1).bit_length() + 8) // 8
    body = v.to_bytes(max(nb, 1), "big", signed=True)
    return b"\x02" + _der_len(len(body)) + body


def _der_seq(body: bytes) -> bytes:
    return b"\x30" + _der_len(len(body)) + body


def _parse_rs(sig: bytes):
    i = 2
    out = []
    for _ in range(2):
        ln = sig[i + 1]
        out.append(int.from_bytes(sig[i + 2:i + 2 + ln], "big", signed=True))
        i += 2 + ln
    return out


def add_ecdsa_adversarial(w: Workload, frac: float = 0.01, seed: int = 7) -> Workload:
    """Mutates a fraction of the ECDSA elements of w uniformly over D1–D8
    (SURVEY §8d).  Signatures that no longer fit sig_stride are left valid."""
    rng = np.random.default_rng(seed)
    ec = np.flatnonzero((w.scheme == 2) | (w.scheme == 3))
    k = int(round(len(ec) * frac))
    idx = rng.choice(ec, size=k, replace=False)
    classes = list(w.classes) if w.classes is not None else ["valid"] * w.n
    for j, i in enumerate(idx):
        cls = EC_CLASSES[j % len(EC_CLASSES)]
        n = _N[int(w.scheme[i])]
        sig = w.sig[i, :w.sig_len[i]].tobytes()
        r, s = _parse_rs(sig)
        new = sig
        if cls == "D1":
            if rng.integers(2):
                b = bytearray(sig); b[6 + rng.integers(len(b) - 6)] ^= 1 << int(rng.integers(8)); new = bytes(b)
            else:
                o = int(w.msg_off[i]); w.msg[o + rng.integers(max(int(w.msg_len[i]), 1))] ^= np.uint8(1)
        elif cls == "D2":
            new = _der_seq(_der_int(0) + _der_int(s)) if rng.integers(2) else _der_seq(_der_int(r) + _der_int(0))
        elif cls == "D3":
            new = _der_seq(_der_int(r + n) + _der_int(s)) if rng.integers(2) else _der_seq(_der_int(r) + _der_int(s + n))
        elif cls == "D4":
            new = _der_seq(_der_int(-r) + _der_int(s))
        elif cls == "D5":
            ri = _der_int(r)
            new = _der_seq(b"\x02" + bytes([ri[1] + 1]) + b"\x00" + ri[2:] + _der_int(s))
        elif cls == "D6":
            body = _der_int(r) + _der_int(s)
            new = b"\x30\x81" + bytes([len(body)]) + body
        elif cls == "D7":
            new = sig + b"\x00"
        elif cls == "D8":
            new = _der_seq(_der_int(r) + _der_int(n - s))
        if len(new) > w.sig_stride:
            continue
        classes[i] = cls
        w.sig[i, :] = 0
        w.sig[i, :len(new)] = np.frombuffer(new, dtype=np.uint8)
        w.sig_len[i] = len(new)
    w.classes = classes
    return w


# ---------------------------------------------------------- config 4 (transactions)
HEADER = b"corda\x00\x00\x01"  # Kryo P2P header (node-api SerializationScheme.kt:216)


class TxWorkload:
    """Config-4 shaped SignedTransaction batch in the cg_tx_verify_batch layout."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _tx_components(n_tx: int, rng, seed: int):
    """Component layout of config-4 transactions (shared by the SignedTransaction and
    the FilteredTransaction workloads)."""
    c = lib()
    n_in = rng.integers(0, 4, n_tx); n_att = rng.integers(0, 2, n_tx); n_out = rng.integers(1, 4, n_tx)
    n_cmd = rng.integers(1, 3, n_tx); has_tw = rng.random(n_tx) < 0.3
    # components in availableComponents order (MerkleTransaction.kt:74-87), vectorized:
    # category c of tx t contributes counts[c][t] leaves; a stable sort by tx keeps
    # the category order inside each tx
    ones = np.ones(n_tx, dtype=np.int64)
    cats = [(n_in, lambda k: rng.integers(48, 65, k)), (n_att, lambda k: np.full(k, 48)),
            (n_out, lambda k: rng.integers(300, 701, k)), (n_cmd, lambda k: rng.integers(150, 301, k)),
            (ones, lambda k: rng.integers(150, 251, k)), (has_tw.astype(np.int64), lambda k: np.full(k, 40)),
            (ones, lambda k: np.full(k, 44))]
    tx_of = np.concatenate([np.repeat(np.arange(n_tx), cnt) for cnt, _ in cats])
    lens_all = np.concatenate([gen(int(cnt.sum())) for cnt, gen in cats])
    order = np.argsort(tx_of, kind="stable")
    comp_len = lens_all[order].astype(np.uint32)
    per_tx = sum(cnt for cnt, _ in cats)
    comp_start = np.zeros(n_tx + 1, dtype=np.uint32)
    comp_start[1:] = np.cumsum(per_tx)
    comp_off = np.zeros(len(comp_len), dtype=np.uint64)
    comp_off[1:] = np.cumsum(comp_len[:-1], dtype=np.uint64)
    arena = np.empty(int(comp_len.sum()) + 1, dtype=np.uint8)
    c.dg_fill_bytes(arena.ctypes.data, len(arena), seed * 1000 + 1)
    # every serialized component starts with the Kryo header
    arena[(comp_off[:, None] + np.arange(8, dtype=np.uint64)).ravel()] = np.tile(
        np.frombuffer(HEADER, dtype=np.uint8), len(comp_off))
    salts = np.empty(32 * n_tx, dtype=np.uint8)
    c.dg_fill_bytes(salts.ctypes.data, len(salts), seed * 1000 + 2)
    return n_in, n_att, n_out, n_cmd, has_tw, arena, comp_off, comp_len, comp_start, salts


def make_tx_batch(n_tx: int, seed: int = 4, key_base: int = 9_000_000, threads: int | None = None,
                  tamper_frac: float = 0.01, key_reuse: int = 0) -> TxWorkload:
    """Trader-demo / loadtest shapes: inputs U{0..3},
    attachments U{0..1}, outputs U{1..3}, commands U{1..2}, notary 1,
    timeWindow p=0.3, salt 1; estimated Kryo sizes; signers = distinct command
    signers (+ notary when inputs > 0 or a time window); schemes 70/15/15 %
    Ed25519/R1/K1; signatures over the tx id; tamper_frac of txs get one leaf byte
    flipped after signing (their id changes, so every signature rejects)."""
    rng = np.random.default_rng(seed)
    c = lib()
    (n_in, n_att, n_out, n_cmd, has_tw, arena, comp_off, comp_len, comp_start,
     salts) = _tx_components(n_tx, rng, seed)
    ids = np.zeros(32 * n_tx, dtype=np.uint8)
    assert c.dg_txid_batch(arena.ctypes.data, comp_off.ctypes.data, comp_len.ctypes.data, comp_start.ctypes.data,
                           salts.ctypes.data, n_tx, ids.ctypes.data) == 0
    n_sig = n_cmd + ((n_in > 0) | has_tw)
    sig_start = np.zeros(n_tx + 1, dtype=np.uint32)
    sig_start[1:] = np.cumsum(n_sig)
    total = int(sig_start[-1])
    scheme = rng.choice(np.array([4, 3, 2], dtype=np.uint8), size=total, p=[0.7, 0.15, 0.15])
    msg_off = np.repeat(np.arange(n_tx, dtype=np.uint64) * 32, n_sig)
    msg_len = np.full(total, 32, dtype=np.uint32)
    pk = np.zeros((total, 64), dtype=np.uint8)
    sig = np.zeros((total, 72), dtype=np.uint8)
    sig_len = np.zeros(total, dtype=np.uint32)
    c.dg_set_key_options(key_reuse, 0)
    rc = c.dg_sign_batch(total, scheme.ctypes.data, key_base, pk.ctypes.data, 64, sig.ctypes.data, 72,
                         sig_len.ctypes.data, ids.ctypes.data, msg_off.ctypes.data, msg_len.ctypes.data,
                         threads or min(16, os.cpu_count() or 1))
    c.dg_set_key_options(0, 0)
    assert rc == 0
    tampered = rng.random(n_tx) < tamper_frac
    for t in np.flatnonzero(tampered):
        c0 = int(comp_start[t])
        arena[int(comp_off[c0]) + 8] ^= 1  # first component, past the header
    return TxWorkload(n_tx=n_tx, arena=arena, comp_off=comp_off, comp_len=comp_len, comp_start=comp_start,
                      salts=salts, ids=ids, sig_start=sig_start, scheme=scheme, pk=pk, sig=sig, sig_len=sig_len,
                      tampered=tampered)


def tile_tx_batch(w: TxWorkload, n_tx: int, tamper_frac: float = 0.01, seed: int = 5) -> TxWorkload:
    """A pool of signed transactions repeated to n_tx (each copy owns its leaf
    bytes), then tamper_frac of the txs get one leaf byte flipped (their id
    changes, so every signature of that tx rejects)."""
    reps = -(-n_tx // w.n_tx)
    a_len = int(w.comp_off[-1]) + int(w.comp_len[-1])
    n_comp = int(w.comp_start[w.n_tx])
    n_sig = int(w.sig_start[w.n_tx])
    arena = np.concatenate([np.tile(w.arena[:a_len], reps), np.zeros(1, np.uint8)])
    comp_off = (w.comp_off[None, :n_comp] + np.arange(reps, dtype=np.uint64)[:, None] * np.uint64(a_len)).ravel()
    comp_len = np.tile(w.comp_len[:n_comp], reps)
    comp_start = np.concatenate([np.zeros(1, np.uint32),
                                 np.cumsum(np.tile(np.diff(w.comp_start), reps), dtype=np.uint64).astype(np.uint32)])
    sig_start = np.concatenate([np.zeros(1, np.uint32),
                                np.cumsum(np.tile(np.diff(w.sig_start), reps), dtype=np.uint64).astype(np.uint32)])
    comp_start, sig_start = comp_start[:n_tx + 1], sig_start[:n_tx + 1]
    nc, ns = int(comp_start[-1]), int(sig_start[-1])
    t = TxWorkload(n_tx=n_tx, arena=arena, comp_off=comp_off[:nc].copy(), comp_len=comp_len[:nc].copy(),
                   comp_start=comp_start, salts=np.tile(w.salts[:32 * w.n_tx], reps)[:32 * n_tx].copy(),
                   ids=np.tile(w.ids[:32 * w.n_tx], reps)[:32 * n_tx].copy(), sig_start=sig_start,
                   scheme=np.tile(w.scheme[:n_sig], reps)[:ns].copy(), pk=np.tile(w.pk[:n_sig], (reps, 1))[:ns].copy(),
                   sig=np.tile(w.sig[:n_sig], (reps, 1))[:ns].copy(), sig_len=np.tile(w.sig_len[:n_sig], reps)[:ns].copy(),
                   tampered=np.zeros(n_tx, dtype=bool))
    rng = np.random.default_rng(seed)
    t.tampered = rng.random(n_tx) < tamper_frac
    first = t.comp_start[:-1][t.tampered]
    t.arena[t.comp_off[first] + 8] ^= 1  # first component, past the Kryo header
    return t


# ------------------------------------------------------------ FilteredTransactions
class FtxWorkload:
    """FilteredTransaction batch in the cg_ftx_verify_batch layout."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _sha256(b: bytes) -> bytes:
    import hashlib
    return hashlib.sha256(b).digest()


def _partial_postorder(leaves: list, include: set) -> list:
    """PartialMerkleTree.build over the full tree of `leaves` (zero-hash padded),
    emitted as the (kind, hash) post-order program; returns (root, program)."""
    level = list(leaves)
    while len(level) & (len(level) - 1):
        level.append(bytes(32))
    # each entry: (hash, has_included, program)
    nodes = [(h, h in include, [(0 if h in include else 1, h)]) for h in level]
    while len(nodes) > 1:
        nxt = []
        for i in range(0, len(nodes), 2):
            (hl, fl, pl), (hr, fr, pr) = nodes[i], nodes[i + 1]
            h = _sha256(hl + hr)
            nxt.append((h, fl or fr, pl + pr + [(2, bytes(32))] if (fl or fr) else [(1, h)]))
        nodes = nxt
    return nodes[0][0], nodes[0][2]


def make_ftx_batch(n_pool: int, seed: int = 11) -> FtxWorkload:
    """What the non-validating notary receives (NotaryFlow.kt:72): each config-4
    transaction filtered to its inputs and time window (transactions with neither
    are not notarised and are skipped), with the nonces of those components and the
    partial Merkle tree over the full tx (PartialMerkleTree.build).  All valid."""
    rng = np.random.default_rng(seed)
    (n_in, n_att, n_out, n_cmd, has_tw, arena, comp_off, comp_len, comp_start,
     salts) = _tx_components(n_pool, rng, seed)
    f_comps, f_nonces, progs, roots = [], [], [], []
    for t in range(n_pool):
        if n_in[t] == 0 and not has_tw[t]:
            continue
        c0, c1 = int(comp_start[t]), int(comp_start[t + 1])
        salt = salts[32 * t:32 * t + 32].tobytes()
        sers = [arena[int(comp_off[c]):int(comp_off[c]) + int(comp_len[c])].tobytes() for c in range(c0, c1)]
        nonces = [_sha256(salt + i.to_bytes(4, "big")) for i in range(len(sers) - 1)]
        leaves = [_sha256(x + n) for x, n in zip(sers, nonces)] + [_sha256(sers[-1])]
        vis = list(range(int(n_in[t])))
        if has_tw[t]:
            vis.append(len(sers) - 2)  # the time window sits just before the salt
        root, prog = _partial_postorder(leaves, {leaves[i] for i in vis})
        f_comps.append([sers[i] for i in vis])
        f_nonces.append([nonces[i] for i in vis])
        progs.append(prog)
        roots.append(root)
    n = len(roots)
    flat = [x for cs in f_comps for x in cs]
    fcl = np.array([len(x) for x in flat], dtype=np.uint32)
    fco = np.zeros(len(flat), dtype=np.uint64)
    fco[1:] = np.cumsum(fcl[:-1], dtype=np.uint64)
    fcs = np.zeros(n + 1, dtype=np.uint32)
    fcs[1:] = np.cumsum([len(cs) for cs in f_comps])
    nst = np.zeros(n + 1, dtype=np.uint32)
    nst[1:] = np.cumsum([len(p) for p in progs])
    return FtxWorkload(
        n=n, arena=np.frombuffer(b"".join(flat) + b"\0", dtype=np.uint8).copy(), comp_off=fco, comp_len=fcl,
        comp_start=fcs, nonces=np.frombuffer(b"".join(x for ns in f_nonces for x in ns), dtype=np.uint8).copy(),
        node_start=nst, node_kind=np.array([k for p in progs for k, _ in p], dtype=np.uint8),
        node_hash=np.frombuffer(b"".join(h for p in progs for _, h in p), dtype=np.uint8).copy(),
        roots=np.frombuffer(b"".join(roots), dtype=np.uint8).copy(), expected=np.zeros(n, dtype=np.uint8))


def tile_ftx_batch(w: FtxWorkload, n: int, adversarial: float = 0.01, seed: int = 12) -> FtxWorkload:
    """The pool repeated to n filtered transactions (each copy owns its bytes), then
    `adversarial` of them broken, split over: a flipped component byte, a flipped
    root byte, a flipped Leaf/IncludedLeaf hash byte in the tree (expected FALSE)."""
    reps = -(-n // w.n)
    a_len = int(w.comp_off[-1]) + int(w.comp_len[-1])
    nc, nn = int(w.comp_start[-1]), int(w.node_start[-1])
    comp_start = np.concatenate([[0], np.cumsum(np.tile(np.diff(w.comp_start), reps), dtype=np.uint64)])
    node_start = np.concatenate([[0], np.cumsum(np.tile(np.diff(w.node_start), reps), dtype=np.uint64)])
    comp_start, node_start = comp_start[:n + 1].astype(np.uint32), node_start[:n + 1].astype(np.uint32)
    tc, tn = int(comp_start[-1]), int(node_start[-1])
    t = FtxWorkload(
        n=n, arena=np.concatenate([np.tile(w.arena[:a_len], reps), np.zeros(1, np.uint8)]),
        comp_off=(w.comp_off[None, :nc] + np.arange(reps, dtype=np.uint64)[:, None] * np.uint64(a_len)).ravel()[:tc],
        comp_len=np.tile(w.comp_len[:nc], reps)[:tc].copy(), comp_start=comp_start,
        nonces=np.tile(w.nonces[:32 * nc], reps)[:32 * tc].copy(), node_start=node_start,
        node_kind=np.tile(w.node_kind[:nn], reps)[:tn].copy(), node_hash=np.tile(w.node_hash[:32 * nn], reps)[:32 * tn].copy(),
        roots=np.tile(w.roots[:32 * w.n], reps)[:32 * n].copy(), expected=np.zeros(n, dtype=np.uint8))
    rng = np.random.default_rng(seed)
    bad = np.flatnonzero(rng.random(n) < adversarial)
    cls = rng.integers(0, 3, len(bad))
    for b, k in zip(bad, cls):
        if k == 0:
            t.arena[int(t.comp_off[t.comp_start[b]]) + 8] ^= 1
        elif k == 1:
            t.roots[32 * b + 5] ^= 1
        else:
            j = next(j for j in range(int(t.node_start[b]), int(t.node_start[b + 1])) if t.node_kind[j] != 2)
            t.node_hash[32 * j + 3] ^= 1
        t.expected[b] = 1
    return t
