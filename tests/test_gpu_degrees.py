"""Any check degree, as the reference allows (decoder.pyx:131-141 sizes its F/B buffer
per check): degrees above the templated range (2..16) run the runtime-degree kernel
with the forward values parked in an HBM scratch (decoder.hip k_check_generic).  Bit
for bit against the oracle for degrees 17, 33, 65, 100 (and 255 on a small code), in
every schedule, plus the node-level surface process_check_node on such checks."""
import numpy as np
import pytest

from conftest import assert_bit_exact

import oracle as O

pytestmark = pytest.mark.gpu


def _code(rng, degrees, V):
    """One check per listed degree (+ degree-3 filler checks), every variable used."""
    degrees = list(degrees)
    E0 = int(sum(degrees))
    extra = max(0, V - E0)
    degrees += [3] * ((extra + 2) // 3)
    deg = np.array(degrees)
    E = int(deg.sum())
    sockets = np.concatenate([np.arange(V), rng.integers(0, V, E - V)])
    rng.shuffle(sockets)
    cid = np.repeat(np.arange(len(deg)), deg)
    return sockets.astype(np.int64), cid.astype(np.int64)


def _frames(rng, orc, B, V, sig=(0.5, 0.9)):
    word = rng.integers(0, 2, (B, V)).astype(np.uint8)
    synd = np.stack([orc.eval_syndrome(w) for w in word])
    s = rng.uniform(*sig, B)[:, None]
    llr = 2 / s ** 2 * ((1 - 2.0 * word) + s * rng.standard_normal((B, V)))
    return llr, synd


@pytest.mark.parametrize("split", [1, 2, 3])
def test_high_degree_checks_vs_oracle(gpu, split):
    import qamr
    rng = np.random.default_rng(17)
    V = 300
    vid, cid = _code(rng, [17, 33, 65, 100, 17, 5, 7], V)
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    llr, synd = _frames(rng, orc, 70, V)
    old = qamr._lib.tune_get("split")
    try:
        qamr._lib.tune_set("split", split)
        s1, i1, f1 = dec.decode_batch(llr, synd, 30)
    finally:
        qamr._lib.tune_set("split", old)
    s2, i2, f2 = orc.decode_batch(llr, synd, 30)
    assert np.array_equal(s1, s2) and np.array_equal(i1, i2)
    assert_bit_exact(f1, f2)


def test_degree_255_and_all_large(gpu):
    """A code made only of large checks (no templated class at all) and one of degree 255."""
    import qamr
    rng = np.random.default_rng(5)
    V = 400
    vid, cid = _code(rng, [255, 40, 40, 40, 24], V)
    keep = cid < 5  # drop the degree-3 filler: only runtime-degree classes
    vid, cid = vid[keep], cid[keep]
    used = np.unique(vid)
    remap = np.full(V, -1, np.int64)
    remap[used] = np.arange(used.size)
    vid = remap[vid]
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    llr, synd = _frames(rng, orc, 64, int(vid.max()) + 1, sig=(0.3, 0.6))
    s1, i1, f1 = dec.decode_batch(llr, synd, 12)
    s2, i2, f2 = orc.decode_batch(llr, synd, 12)
    assert np.array_equal(s1, s2) and np.array_equal(i1, i2)
    assert_bit_exact(f1, f2)


def test_process_check_node_high_degree(gpu):
    import qamr
    rng = np.random.default_rng(3)
    V = 250
    vid, cid = _code(rng, [100, 65, 33, 17], V)
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    E = vid.size
    C = int(cid.max()) + 1
    synd = rng.integers(0, 2, C).astype(np.uint8)
    for c in range(4):
        v2c = rng.standard_normal(E) * rng.choice([0.5, 3.0, 20.0], E)
        c1 = rng.standard_normal(E)
        c2 = c1.copy()
        dec.process_check_node(c, synd, c1, v2c)
        orc.process_check_node(c, synd, c2, v2c)
        assert_bit_exact(c1, c2)
