"""Wire codec: the reference's Data.Binary payloads of
ClientRequest / ServerResponse (Common.hs:24,47,55).

CPU tests pin the oracle (oracle/wire_ref.py) to hand-derived byte vectors
from binary-0.8.5.1's generic encoding; GPU tests check the HIP codec against
the oracle byte for byte (encode) and value for value (decode), including
malformed records.  The reference cannot run here (no GHC), so the vectors
are derived from the published algorithm, not captured from a live node."""
import numpy as np
import pytest

import pxb
import wire_ref as W


def be(v):
    return v.to_bytes(8, "big", signed=True)


# ---- oracle known answers ---------------------------------------------------------
def test_request_vectors():
    # AskForTicket (Ticket 1): tag 0, Int64 BE
    assert W.encode((W.ASK, 1, 0, 0), W.REQUEST) == b"\x00" + be(1)
    # Propose (Ticket 1, "c1.1"): tag 1, Ticket, String length 4, "c1.1"
    assert W.encode((W.PROPOSE, 1, 0, (1 << 24) | 1), W.REQUEST) == b"\x01" + be(1) + be(4) + b"c1.1"
    # Execute (Ticket 300)
    assert W.encode((W.EXECUTE, 300, 0, 0), W.REQUEST) == b"\x02" + be(300)
    # a negative Int is two's complement (Ticket is Int)
    assert W.encode((W.ASK, -2, 0, 0), W.REQUEST) == b"\x00" + b"\xff" * 7 + b"\xfe"


def test_response_vectors():
    # Round1OK (Ticket 2) Nothing
    assert W.encode((W.R1OK, 2, 0, 0), W.RESPONSE) == b"\x00" + be(2) + b"\x00"
    # Round1OK (Ticket 3) (Just (Ticket 2, "c12.345"))
    assert W.encode((W.R1OK, 3, 2, (12 << 24) | 345), W.RESPONSE) == \
        b"\x00" + be(3) + b"\x01" + be(2) + be(7) + b"c12.345"
    assert W.encode((W.HAVE, 9, 0, 0), W.RESPONSE) == b"\x01" + be(9)
    assert W.encode((W.R2S, 0, 0, 0), W.RESPONSE) == b"\x02"


def test_oracle_round_trip_and_errors():
    rng = np.random.default_rng(1)
    for kind in (W.REQUEST, W.RESPONSE):
        for _ in range(500):
            m = _random_msg(rng, kind)
            st, d = W.decode(W.encode(m, kind), kind)
            assert st == W.OK and d == m
    bad = [
        (b"", W.REQUEST, W.E_LENGTH), (b"\x03" + be(1), W.REQUEST, W.E_TAG),
        (b"\x00" + be(1)[:5], W.REQUEST, W.E_LENGTH), (b"\x00" + be(1) + b"\x00", W.REQUEST, W.E_LENGTH),
        (b"\x00" + be(1 << 40), W.REQUEST, W.E_RANGE),
        (b"\x01" + be(1) + be(4) + b"d1.1", W.REQUEST, W.E_STRING),
        (b"\x01" + be(1) + be(5) + b"c01.1", W.REQUEST, W.E_STRING),
        (b"\x01" + be(1) + be(4) + b"c1..", W.REQUEST, W.E_STRING),
        (b"\x01" + be(1) + be(3) + b"c11", W.REQUEST, W.E_STRING),
        (b"\x01" + be(1) + be(6) + b"c256.1", W.REQUEST, W.E_RANGE),
        (b"\x01" + be(1) + be(8) + b"c1.1", W.REQUEST, W.E_LENGTH),
        (b"\x00" + be(1) + b"\x02", W.RESPONSE, W.E_TAG),
        (b"\x05", W.RESPONSE, W.E_TAG), (b"\x02\x00", W.RESPONSE, W.E_LENGTH),
    ]
    for data, kind, want in bad:
        assert W.decode(data, kind)[0] == want, (data, kind)


def _random_msg(rng, kind):
    tag = int(rng.integers(0, 3))
    x = int(rng.integers(-5, 1 << 14))
    code = (int(rng.integers(0, 256)) << 24) | int(rng.integers(0, 1 << 24))
    if kind == W.REQUEST:
        return (tag, x, 0, code if tag == W.PROPOSE else 0)
    if tag == W.R1OK:
        has = rng.random() < 0.6 and code != 0
        return (tag, x, int(rng.integers(0, 1 << 14)) if has else 0, code if has else 0)
    return (tag, x if tag == W.HAVE else 0, 0, 0)


def _batch(kind, n, seed):
    rng = np.random.default_rng(seed)
    return np.array([_random_msg(rng, kind) for _ in range(n)], dtype=np.int64).astype(np.uint32)


def _as_msg(row):
    """uint32 pxb_msg row -> (tag, x, y, z) with signed tickets, unsigned command."""
    sx = row.astype(np.int32)
    return (int(row[0]), int(sx[1]), int(sx[2]), int(row[3]))


# ---- GPU codec == oracle ----------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("kind", [W.REQUEST, W.RESPONSE])
def test_gpu_encode_matches_oracle(gpu_lib, kind):
    msgs = _batch(kind, 20000, 7 + kind)
    data, offs = pxb.wire_encode(msgs, kind)
    want, woffs = W.encode_batch([_as_msg(m) for m in msgs], kind)
    assert list(offs) == woffs
    assert data == want


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [W.REQUEST, W.RESPONSE])
def test_gpu_decode_round_trip(gpu_lib, kind):
    msgs = _batch(kind, 20000, 11 + kind)
    data, offs = pxb.wire_encode(msgs, kind)
    back, st = pxb.wire_decode(data, offs, kind)
    assert (st == W.OK).all()
    assert np.array_equal(back, msgs)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [W.REQUEST, W.RESPONSE])
def test_gpu_decode_malformed_matches_oracle(gpu_lib, kind):
    """Random corruptions of valid records (byte flips, truncation, trailing
    bytes): the GPU status and values equal the oracle's."""
    rng = np.random.default_rng(3 + kind)
    msgs = _batch(kind, 3000, 5 + kind)
    recs = [W.encode(_as_msg(m), kind) for m in msgs]
    bad = []
    for r in recs:
        r = bytearray(r)
        op = rng.integers(0, 4)
        if op == 0 and len(r) > 1:
            r = r[:int(rng.integers(0, len(r)))]
        elif op == 1:
            r += bytes([int(rng.integers(0, 256))])
        elif op == 2:
            i = int(rng.integers(0, len(r)))
            r[i] = int(rng.integers(0, 256))
        bad.append(bytes(r))
    offs = np.cumsum([0] + [len(r) for r in bad]).astype(np.uint64)
    got, st = pxb.wire_decode(b"".join(bad), offs, kind)
    for i, r in enumerate(bad):
        ws, wm = W.decode(r, kind)
        assert st[i] == ws, (i, r, st[i], ws)
        if ws == W.OK:
            assert _as_msg(got[i]) == wm


@pytest.mark.gpu
def test_gpu_wire_empty_batch(gpu_lib):
    data, offs = pxb.wire_encode(np.zeros((0, 4), np.uint32), W.REQUEST)
    assert data == b"" and list(offs) == [0]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [W.REQUEST, W.RESPONSE])
def test_gpu_decode_irregular_offsets_matches_oracle(gpu_lib, kind):
    """Offsets that are not a clean framing: decreasing pairs (an empty record),
    a tile whose range runs backwards, a tile whose range exceeds the LDS stage.
    Every record i is bytes[offs[i]:max(offs[i], offs[i+1])], as in the oracle;
    such tiles are parsed from HBM instead of the LDS stage.  Offsets past the
    end of the buffer make a length error and are never read."""
    rng = np.random.default_rng(21 + kind)
    msgs = _batch(kind, 5000, 17 + kind)
    data, offs = pxb.wire_encode(msgs, kind)
    offs = np.array(offs, dtype=np.uint64)
    total = int(offs[-1])
    for i in rng.choice(np.arange(1, 5000), 40, replace=False):
        offs[i] = int(rng.integers(0, total + 1))       # random framing errors
    offs[1024] = total                                   # tile 0 too long, tile 1 backwards
    offs[3000] = 0
    for i in rng.choice(np.arange(1, 5000), 12, replace=False):
        offs[i] = total + int(rng.integers(1, 1 << 20))  # past the end of the buffer
    offs[-1] = total + 7
    got, st = pxb.wire_decode(data, offs, kind)
    for i in range(5000):
        b, e = int(offs[i]), int(offs[i + 1])
        ws, wm = W.decode_at(data, b, e, kind)
        assert st[i] == ws, (i, b, e, st[i], ws)
        if ws == W.OK:
            assert _as_msg(got[i]) == wm


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [W.REQUEST, W.RESPONSE])
@pytest.mark.parametrize("n", [1, 255, 256, 257, 20000])
def test_gpu_encode_all_matches_oracle(gpu_lib, kind, n):
    """pxb_wire_encode_all (fused size + encode, device buffers) == the oracle,
    including ragged last tiles."""
    import torch
    msgs = _batch(kind, n, 31 + kind + n)
    d_m = torch.from_numpy(msgs.view(np.int32)).cuda()
    d_o = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
    d_b = torch.zeros(n * pxb.WIRE_MAX_BYTES, dtype=torch.uint8, device="cuda")
    pxb.wire_encode_device(d_m, kind, d_o, d_b)
    torch.cuda.synchronize()
    offs = d_o.cpu().numpy().astype(np.uint64)
    want, woffs = W.encode_batch([_as_msg(m) for m in msgs], kind)
    assert list(offs) == woffs
    assert d_b[:len(want)].cpu().numpy().tobytes() == want


def _batch_fast(kind, n, seed):
    """Vectorised random records (the bench's mix plus requests), for sizes the
    per-record generator above is too slow for."""
    rng = np.random.default_rng(seed)
    tag = rng.integers(0, 3, n).astype(np.uint32)
    m = np.zeros((n, 4), np.uint32)
    m[:, 0] = tag
    x = rng.integers(-5, 1 << 14, n).astype(np.int64).astype(np.uint32)
    code = ((rng.integers(1, 256, n) << 24) | rng.integers(0, 1 << 24, n)).astype(np.uint32)
    if kind == W.REQUEST:
        m[:, 1] = x
        m[:, 3] = np.where(tag == W.PROPOSE, code, 0)
    else:
        just = (tag == W.R1OK) & (rng.random(n) < 0.6)
        m[:, 1] = np.where(tag == 2, 0, x)
        m[:, 2] = np.where(just, rng.integers(0, 1 << 14, n), 0)
        m[:, 3] = np.where(just, code, 0)
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [W.REQUEST, W.RESPONSE])
def test_gpu_encode_all_at_scale_on_two_streams(gpu_lib, kind):
    """pxb_wire_encode_all (tile sums, their scan, encode) equals the two-pass
    size scan + encode (pxb_wire_size, pxb_wire_encode) at 2^22 + 17 messages,
    on two streams at once with different batches, three times over: each
    call's scratch (tile sums, tile offsets, scan storage) is its own,
    allocated and freed on its stream."""
    import torch
    n = (1 << 22) + 17
    batches = [_batch_fast(kind, n, 90 + kind), _batch_fast(kind, n, 91 + kind)]
    want = [pxb.wire_encode(b, kind) for b in batches]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = []
    for b, st in zip(batches, streams):
        d_m = torch.from_numpy(b.view(np.int32)).cuda()
        d_o = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
        d_b = torch.zeros(n * pxb.WIRE_MAX_BYTES, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        bufs.append((d_m, d_o, d_b, st))
    for _ in range(3):                                  # (repeated: the pool's buffers are reused)
        for d_m, d_o, d_b, st in bufs:
            pxb.wire_encode_device(d_m, kind, d_o, d_b, stream=st.cuda_stream)
    torch.cuda.synchronize()
    for (data, offs), (_, d_o, d_b, _) in zip(want, bufs):
        got_offs = d_o.cpu().numpy().astype(np.uint64)
        assert np.array_equal(got_offs, offs)
        assert d_b[:len(data)].cpu().numpy().tobytes() == data
