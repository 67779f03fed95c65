"""CPU: the C-ABI library loads, exports every symbol include/onitama_az.h declares, and its
host-side logic (tables, deals, weights layout, test evaluator) matches the oracle. No GPU
compute is called here."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from onitama_az import _abi
from onitama_az import weights as W

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "onitama_az.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(oaz_[a-z0-9_]+)\s*\(", text)))


def test_header_functions_exported(lib):
    names = declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_abi.EXPORTED_SYMBOLS), set(names) ^ set(_abi.EXPORTED_SYMBOLS)


def test_abi_version_and_structs(lib):
    assert lib.oaz_abi_version() == _abi.ABI_VERSION == 5
    assert C.sizeof(_abi.oaz_config) == 120 and _abi.oaz_config.search_time_ns.offset == 104
    assert C.sizeof(_abi.oaz_comm_stats) == 56


def test_default_config_matches_reference_train_bin():  # bin/train.rs:50-78
    c = _abi.default_config()
    assert (c.blocks, c.channels, c.in_planes, c.sims, c.c_puct, c.train_noise, c.max_plies) == (5, 64, 21, 400, 5.0, 1, 150)
    assert c.dirichlet_alpha == 0.03 and c.dirichlet_eps == 0.25


def test_attack_maps_equal_oracle(lib, orc):
    am = np.zeros((2, 16, 25), dtype=np.uint32)
    lib.oaz_attack_maps(_abi.ptr(am))
    assert np.array_equal(am, orc.attack_maps())


def test_deal_and_initial_state_equal_oracle(lib, orc):
    for gid in list(range(200)) + [2**40 + 5]:
        d = (C.c_uint8 * 5)()
        lib.oaz_deal_deck(C.c_uint64(123), C.c_uint64(gid), d)
        assert list(d) == list(orc.deal_deck(123, gid))
        assert len(set(d)) == 5
        a = np.zeros(1, dtype=_abi.STATE_DTYPE)
        lib.oaz_initial_state(d, _abi.ptr(a))
        assert a.tobytes() == orc.initial_state(np.array(list(d), np.uint8)).tobytes()


def test_hash_eval_equal_oracle(lib, orc):
    from conftest import random_positions
    for s in random_positions(orc, 100, seed=4):
        s = s.reshape(1).copy()
        p, v = np.zeros(50, np.float32), np.zeros(1, np.float32)
        lib.oaz_hash_eval(_abi.ptr(s), _abi.ptr(p), _abi.ptr(v))
        p2, v2 = orc.hash_eval(s)
        assert np.array_equal(p, p2) and v[0] == v2


@pytest.mark.parametrize("blocks", [0, 3, 5, 6])
def test_weight_layout(lib, orc, blocks):
    n = lib.oaz_weight_count(blocks, 64, 21)
    assert n == W.weight_count(blocks) == orc.load().orc_weight_count(blocks)
    w = W.random_weights(7, blocks)
    named = W.named_from_blob(w, blocks)
    assert np.all(named["bn1|weight"] == 1) and np.all(named["bn1|running_var"] == 1)
    assert np.all(np.abs(named["conv_init_1|weight"]) <= 1 / np.sqrt(21 * 9))
    assert np.array_equal(W.blob_from_named(named, blocks), w)


def test_param_counts_match_survey():
    assert W.weight_count(3) == 240_006 and W.weight_count(5) == 388_742 and W.weight_count(6) == 463_110


@pytest.mark.skipif(not Path("/root/reference/models/model_5e-3_3_resnet.ot").exists(), reason="reference not mounted")
def test_ot_reader_matches_committed_fixture(trained3):
    named = W.read_ot("/root/reference/models/model_5e-3_3_resnet.ot")
    assert W.blocks_from_names(named) == 3 and len(named) == 60
    assert np.array_equal(W.blob_from_named(named, 3), trained3)


REF_MODELS = sorted(Path("/root/reference/models").glob("*.ot")) if Path("/root/reference/models").exists() else []


@pytest.mark.skipif(not REF_MODELS, reason="reference not mounted")
@pytest.mark.parametrize("path", REF_MODELS, ids=lambda p: p.name)
def test_c_ot_reader_on_reference_archives(path):
    """The library's C reader (oaz_ot_read, the product path of from_model_file) reads every .ot the
    reference ships (libtorch-written archives: BINPUT memo, NEWOBJ module, FB-padded members)
    exactly as the Python restatement does."""
    blob, blocks = W.ot_blob(str(path))
    named = W.read_ot(str(path))
    assert blocks == W.blocks_from_names(named)
    assert np.array_equal(blob, W.blob_from_named(named, blocks))


def test_c_ot_reader_and_named_loader(trained3, tmp_path):
    """oaz_ot_read on an archive written with the tensors in a non-canonical order; the named loader
    (oaz_weights_from_named) with tch's '.' separator and shuffled order; its refusals (Q13)."""
    named = W.named_from_blob(trained3, 3)
    p = tmp_path / "m.ot"
    W.write_ot(str(p), {k: named[k] for k in sorted(named, reverse=True)})
    blob, blocks = W.ot_blob(str(p))
    assert blocks == 3 and np.array_equal(blob, trained3)
    table = W.tensor_table(3)
    assert [(n, int(np.prod(s))) for n, s in W.canonical_layout(3)] == table
    rng = np.random.default_rng(0)
    keys = list(named)
    rng.shuffle(keys)
    dotted = {k.replace("|", "."): named[k] for k in keys}
    assert np.array_equal(W.blob_from_named_c(dotted, 3), trained3)
    for bad, msg in ((dict(list(dotted.items())[1:]), "missing"),
                     (dict(dotted, **{"extra|weight": np.zeros(3, np.float32)}), "not part of"),
                     (dict(dotted, **{"bn1.weight": np.zeros(65, np.float32)}), "elements")):
        with pytest.raises(_abi.OazError, match=msg):
            W.blob_from_named_c(bad, 3)
    with pytest.raises(_abi.OazError, match="cannot open"):
        W.ot_blob(str(tmp_path / "absent.ot"))
    (tmp_path / "junk.ot").write_bytes(b"not a zip archive at all" * 10)
    with pytest.raises(_abi.OazError, match="zip"):
        W.ot_blob(str(tmp_path / "junk.ot"))


def test_c_ot_reader_survives_corrupt_archives(trained3, tmp_path):
    """The C reader takes an untrusted file: truncations and byte mutations of a valid archive
    (offsets, sizes, pickle opcodes, shapes) must end in OAZ_ERR_WEIGHTS or a correct read, never a
    crash (this process would die) or a silently different blob."""
    p = tmp_path / "m.ot"
    W.write_ot(str(p), W.named_from_blob(trained3, 3))
    good = p.read_bytes()
    rng = np.random.default_rng(7)
    q = tmp_path / "bad.ot"
    cases = [good[:k] for k in (0, 21, 22, 100, len(good) // 2, len(good) - 23, len(good) - 1)]
    for _ in range(300):
        b = bytearray(good)
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, len(b)))
            if rng.random() < 0.5:  # near the directory / pickle (most structure lives there)
                i = len(b) - 1 - int(rng.integers(0, min(len(b), 4096)))
            b[i] = int(rng.integers(0, 256))
        cases.append(bytes(b))
    ok = 0
    for data in cases:
        q.write_bytes(data)
        try:
            blob, blocks = W.ot_blob(str(q))
        except _abi.OazError:
            continue
        ok += 1  # a mutation inside tensor bytes reads fine; anything else must still be the network
        assert blocks == 3 and blob.shape == trained3.shape
    assert ok < len(cases)


def test_ot_writer_round_trip(trained3, tmp_path):
    """save_vs format (train.rs:414-430): read back by the safe reader and by TorchScript's own
    loader (the loader tch's VarStore::load drives), tensors stored 64-byte aligned."""
    import struct
    import zipfile
    p = W.checkpoint_path(str(tmp_path), 7, True, "20260101_120000")
    assert p.endswith("/best_model_7_20260101_120000.ot")
    W.save_blob_ot(p, trained3, 3)
    assert np.array_equal(W.blob_from_named(W.read_ot(p), 3), trained3)
    raw = open(p, "rb").read()
    z = zipfile.ZipFile(p)
    assert z.testzip() is None
    for info in z.infolist():
        if "/data/" in info.filename:
            n, e = struct.unpack("<HH", raw[info.header_offset + 26: info.header_offset + 30])
            assert (info.header_offset + 30 + n + e) % 64 == 0
    import torch
    m = torch.jit.load(p)
    params = dict(m.named_parameters())
    named = W.named_from_blob(trained3, 3)
    assert set(params) == set(named)
    for k, v in named.items():
        assert np.array_equal(params[k].detach().numpy(), v), k


def test_c_ot_writer_bytes_equal_python_writer(tmp_path):
    """oaz_ot_write (the product writer, C) emits byte for byte the archive the independent Python
    restatement (weights.write_ot over Python's zipfile) writes for the same tensors, for 0, 3 and 5
    blocks, and both readers read it back bit-equal (save_vs, train.rs:414-430)."""
    for blocks, blob in ((0, W.random_weights(3, 0)),
                         (3, np.load(ROOT / "tests/golden/weights_3block_trained.npy")),
                         (5, np.load(ROOT / "tests/golden/weights_5block_trained.npy"))):
        c_path, py_dir = tmp_path / f"model_{blocks}_20260101_120000.ot", tmp_path / f"py{blocks}"
        py_dir.mkdir()
        W.save_blob_ot(str(c_path), blob, blocks)
        W.write_ot(str(py_dir / c_path.name), W.named_from_blob(blob, blocks))
        assert c_path.read_bytes() == (py_dir / c_path.name).read_bytes(), blocks
        got, b = W.ot_blob(str(c_path))
        assert b == blocks and np.array_equal(got, blob)
        assert np.array_equal(W.blob_from_named(W.read_ot(str(c_path)), blocks), blob)
        assert not (tmp_path / (c_path.name + ".tmp")).exists()
    with pytest.raises(_abi.OazError, match="floats given"):
        W.save_blob_ot(str(tmp_path / "bad.ot"), np.zeros(5, np.float32), 3)
    with pytest.raises(_abi.OazError, match="cannot create"):
        W.save_blob_ot(str(tmp_path / "no" / "such" / "dir.ot"), W.random_weights(3, 0), 0)


def _pickle_archive(path, pkl: bytes):
    """A zip whose only member is data.pkl = pkl (stored), as VarStore archives hold it."""
    z = W._AlignedZip(str(path))
    z.add("m/data.pkl", pkl)
    z.close()


def test_ot_readers_bounded_on_crafted_pickles(tmp_path):
    """Crafted data.pkl inputs that alias containers through the memo: a list appended
    to itself, a 64-level doubling DAG (2^64 paths for a tree walk), a 200 000-deep chain of nested
    lists, and a two-list cycle. The C reader refuses or reads them in bounded time and memory
    (index arena, visited set, explicit stack: no exponential walk, no recursive destructor, no
    leaked cycle), ending in OAZ_ERR_WEIGHTS; the Python reader terminates too."""
    import time
    cases = {
        "self_append": b"\x80\x02]q\x00h\x00ah\x00a.",
        "doubling_dag": b"\x80\x02]r\x00\x00\x00\x00" + b"".join(
            b"]r" + k.to_bytes(4, "little") + (b"j" + (k - 1).to_bytes(4, "little") + b"a") * 2
            for k in range(1, 65)) + b".",
        "deep_chain": b"\x80\x02" + b"]" * 200_000 + b"a" * 199_999 + b".",
        "two_cycle": b"\x80\x02]q\x00]q\x01h\x00ah\x01a.",
        "self_setitem": b"\x80\x02}q\x00X\x01\x00\x00\x00kh\x00s.",
    }
    for name, pkl in cases.items():
        p = tmp_path / f"{name}.ot"
        _pickle_archive(p, pkl)
        t0 = time.perf_counter()
        with pytest.raises(_abi.OazError):
            W.ot_blob(str(p))
        assert time.perf_counter() - t0 < 5.0, name
        if name != "deep_chain":  # pickletools' genops walk of 400k opcodes is merely slow
            try:
                W.read_ot(str(p))
            except (ValueError, KeyError, IndexError, AttributeError, TypeError):
                pass
    with pytest.raises(_abi.OazError, match="APPEND"):  # the direct self-reference is refused by name
        W.ot_blob(str(tmp_path / "self_append.ot"))
    # container items up to one below the reader's cap (2^20) through APPENDS, then a TUPLE3 that would
    # cross it: refused there (before ADVICE r4 TUPLE1..3 skipped the cap check, so the count passed the
    # cap and every later check's unsigned subtraction wrapped, turning the cap off)
    cap, chunk = 1 << 20, 65000
    body = [b"\x80\x02Nq\x00]q\x01"]
    left = cap - 1
    while left:
        k = min(chunk, left)
        body.append(b"(" + b"h\x00" * k + b"e")
        left -= k
    body.append(b"h\x00h\x00h\x00\x87(" + b"h\x00" * 10 + b"e.")
    p = tmp_path / "tuple3_over_cap.ot"
    _pickle_archive(p, b"".join(body))
    with pytest.raises(_abi.OazError, match="TUPLEn"):
        W.ot_blob(str(p))


def test_no_device_is_a_loud_error(lib):
    if _abi.device_count() > 0:
        pytest.skip("a GPU is visible")
    cfg = _abi.default_config()
    assert not lib.oaz_create(C.byref(cfg), 0)
    assert b"device" in lib.oaz_last_error()
    s = np.zeros(1, dtype=_abi.STATE_DTYPE)
    assert lib.oaz_movegen(_abi.ptr(s), 1, None, None, None) == -2  # OAZ_ERR_NO_DEVICE, no CPU fallback


def test_display_kat(kats):  # state.rs:397-417 (State::display is host-side formatting)
    from onitama_az.game import ORIGINAL_CARDS, Deck, State
    st = State.with_deck(Deck([ORIGINAL_CARDS[i] for i in range(5)]))
    assert st.display() == kats["display"]["expected"]


def test_root_noise_host_matches_oracle_and_distribution():
    """The engine's root-noise draw (f64 log-domain Beta(alpha, (K-1) alpha), the marginal of the
    reference's per-comparison f64 Dirichlet sample, mcts_arena.rs:186-203) equals the oracle's
    restatement bit for bit, and its sample mean is 1/K (Beta(a, b) mean a / (a + b))."""
    import oracle_ffi as orc
    lib = _abi.load()
    olib = orc.load()
    rng = np.random.default_rng(5)
    for _ in range(2000):
        seed, gid = int(rng.integers(0, 2**63)), int(rng.integers(0, 2**40))
        ply, sim, draw, K = int(rng.integers(0, 152)), int(rng.integers(0, 800)), int(rng.integers(2, 80)), int(rng.integers(2, 41))
        a = lib.oaz_root_noise(seed, gid, ply, sim, draw, 0.03, K)
        b = olib.orc_root_noise(seed, gid, (ply << 16) | sim, draw, 0.03, K)
        assert a == b  # the same f64 value (exact double equality)
        assert 0.0 <= a <= 1.0
    for K in (2, 12, 40):
        xs = np.array([lib.oaz_root_noise(7, g, 0, s, 3, 0.03, K) for g in range(40) for s in range(100)])
        var = (1.0 / K) * (1 - 1.0 / K) / (0.03 * K + 1)  # Beta(a, b) variance, a + b = 0.03 K
        se = np.sqrt(var / len(xs))
        assert abs(xs.mean() - 1.0 / K) < 5 * se, (K, xs.mean())
        assert abs(xs.var() / var - 1.0) < 0.2, (K, xs.var(), var)


def test_root_noise_distribution_ks():
    """The root-noise draw against its target law, Beta(alpha, (K - 1) alpha) — the marginal of one
    component of the reference's f64 Dirichlet(alpha; K) sample (rand_distr 0.4.3, mcts_arena.rs:190-203)
    — with 2 * 10^5 host draws per K (bit-identical to the device's, test above and the noise-on tree
    tests): a Kolmogorov-Smirnov distance and the mass at quantiles 1 % ... 99 % and in the tails.
    The draw is f64, so the law is resolved to within f64's spacing of 1: a draw is 1.0 exactly only
    when 1 - eta < 2^-53 (Y / X below f64's epsilon, where the reference's X / (X + Y) in f64 is 1.0 as
    well: ~16 % of the mass at K = 2; the previous f32 draw collapsed everything within 6e-8 of 1, 30 %).
    The masses between 1 - 1e-7 and 1 - 1e-15, which an f32 draw cannot resolve, are compared one decade
    at a time, the mass at exactly 1.0 as a whole, and the KS sup runs over x < 1 - 2^-52 (a sup over a
    subset: the full-sample Kolmogorov null is conservative for it). Below 1e-300 the mass is < 1e-9."""
    from scipy import stats
    lib = _abi.load()
    x1, n = 1.0 - 2.0 ** -52, 200_000
    for K in (2, 14, 40):
        a, b = 0.03, 0.03 * (K - 1)
        law, flip = stats.beta(a, b), stats.beta(b, a)  # flip: 1 - eta, for the tail near 1
        xs = np.sort(np.array([lib.oaz_root_noise(11, g, 0, s, 5, 0.03, K) for g in range(2000) for s in range(100)]))
        assert xs.dtype == np.float64 and xs.min() >= 0.0 and xs.max() <= 1.0
        assert np.mean(xs <= 1e-300) < 1e-4
        f1, m1 = flip.cdf(1.0 - x1), float(np.mean(xs >= x1))  # the draws that are 1.0 (or 1 - 2^-53)
        assert abs(m1 - f1) < 5 * np.sqrt(max(f1 * (1 - f1), 1.0 / n) / n), (K, m1, f1)
        for lo, hi in ((1e-15, 1e-13), (1e-13, 1e-11), (1e-11, 1e-9), (1e-9, 1e-7)):  # 1 - eta in [lo, hi)
            p = flip.cdf(hi) - flip.cdf(lo)
            m = float(np.mean((1.0 - xs >= lo) & (1.0 - xs < hi)))
            assert abs(m - p) < 5 * np.sqrt(max(p * (1 - p), 1.0 / n) / n), (K, lo, hi, m, p)
        mid = xs[xs < x1]  # KS distance over x < 1 - 2^-52
        lo = np.searchsorted(xs, mid, side="left") / n  # ECDF just below each value
        hi = np.searchsorted(xs, mid, side="right") / n  # ECDF at each value
        F = law.cdf(mid)
        d = float(max(np.max(hi - F), np.max(F - lo)))
        p = float(stats.kstwo(n).sf(d))
        print(f"K={K}: mass at 1.0 {m1:.4f} (law {f1:.4f}); KS D={d:.5f} p={p:.3f}")
        assert p > 1e-3, (K, d, p)
        for q in (0.01, 0.05, 0.25, 0.5, 0.75, 0.95, 0.99):
            xq = law.ppf(q)
            if not xq < x1:
                continue  # inside the mass at 1.0, checked above
            frac = float(np.mean(xs <= xq))
            assert abs(frac - q) < 5 * np.sqrt(q * (1 - q) / n), (K, q, frac)


@pytest.mark.parametrize("kw", [dict(compact=3), dict(compact=-1), dict(parts=3), dict(parts=-1)])
def test_config_compact_and_parts_out_of_range_are_errors(kw):
    """oaz_config.compact is 0, 1 or 2 and parts 0, 1, 2 or 4; anything else fails oaz_create
    before any device work."""
    from onitama_az.engine import Engine
    with pytest.raises(_abi.OazError, match="config out of range"):
        Engine(games=4, sims=4, **kw)
