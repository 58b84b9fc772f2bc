"""The C ABI library without a GPU: it loads, exports every symbol include/cfsec.h
declares, and its host-side logic (matrices, argument checks, Split/Join, code-mode
table, AZ layouts) matches the reference.  No compute call runs here."""
import ctypes
import io
import os
import re

import numpy as np
import pytest

from chubaofs_amd import _lib, codemode as cm
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cfsec.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cfsec_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table out of sync with include/cfsec.h"


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_status_names_match_go_sentinels():
    L = _lib.lib()
    names = {i: L.cfsec_status_name(i).decode() for i in range(15)}
    assert names[1] == "ErrTooFewShards" and names[3] == "ErrShardSize" and names[9] == "ErrInvalidCodeMode"
    assert names[10] == "ErrVerify" and names[11] == "ErrInvalidShards" and names[8] == "errSingular"


@pytest.mark.parametrize("k,m", [(6, 6), (12, 4), (6, 10), (8, 1), (16, 20), (18, 1), (15, 12), (10, 4),
                                 (1, 1), (200, 56)])
def test_engine_matrix_equals_oracle(k, m):
    from chubaofs_amd import reedsolomon
    e = reedsolomon.New(k, m)
    assert np.array_equal(e.matrix(), O.build_matrix(k, k + m))


def test_new_errors():
    from chubaofs_amd import reedsolomon
    with pytest.raises(_lib.ErrInvShardNum):
        reedsolomon.New(0, 4)
    with pytest.raises(_lib.ErrInvShardNum):
        reedsolomon.New(4, -1)
    with pytest.raises(_lib.ErrNotSupported):  # >256 shards is leopard GF16 in the reference
        reedsolomon.New(200, 100)


def test_argument_errors_precede_device_use():
    """checkShards / shard-count checks fire before any device work (KRS/reedsolomon.go)."""
    from chubaofs_amd import reedsolomon
    e = reedsolomon.New(6, 3)
    sh = [np.ones(8, np.uint8) for _ in range(9)]
    with pytest.raises(_lib.ErrTooFewShards):
        e.Encode(sh[:8])
    bad = list(sh)
    bad[2] = np.ones(7, np.uint8)
    with pytest.raises(_lib.ErrShardSize):
        e.Encode(bad)
    with pytest.raises(_lib.ErrShardNoData):
        e.Encode([np.zeros(0, np.uint8)] * 9)
    with pytest.raises(_lib.ErrTooFewShards):
        e.Verify(sh[:3])
    miss = list(sh)
    for i in range(4):
        miss[i] = miss[i][:0]
    with pytest.raises(_lib.ErrTooFewShards):
        e.Reconstruct(miss)
    # all present: Reconstruct is a no-op, no device needed
    e.Reconstruct(list(sh))


def py_split(k, total, data, length):
    """KRS/reedsolomon.go:1574-1632 restated for host buffers (data.size = cap)."""
    per = (length + k - 1) // k
    need = total * per
    buf = data
    eff = length
    if data.size > length:
        eff = min(data.size, need)
        buf[length:eff] = 0
    full = min(eff // per, total)
    out = [bytes(buf[i * per:(i + 1) * per]) for i in range(full)]
    pad = np.zeros((total - full) * per, np.uint8)
    tail = buf[per * full:length]
    pad[:tail.size] = tail
    out += [bytes(pad[j * per:(j + 1) * per]) for j in range(total - full)]
    return out


@pytest.mark.parametrize("k,m,length,cap", [(6, 6, 11, 11), (12, 4, 1000, 1003), (4, 2, 130, 140), (3, 3, 1, 1),
                                           (12, 4, 4096, 8192)])
def test_split_views_caps_and_padding_layout(k, m, length, cap):
    """cfsec_rs_split's shard headers as the reference builds them: data shards data[:per:per], padding
    shards from AllocAligned(npad, per) (KRS/unsafe.go:17-41) -- a 64-byte aligned start, a stride and
    capacity of per rounded up to 64 -- with the partial tail copied shard by shard; pad_needed covers
    the alignment slack."""
    import ctypes
    from chubaofs_amd import reedsolomon
    e = reedsolomon.New(k, m)
    tot = k + m
    data = np.random.default_rng(length + cap).integers(0, 256, cap, dtype=np.uint8)
    ref = data.copy()
    out = (_lib.Shard * tot)()
    need = ctypes.c_size_t(0)
    L = e._L
    st = L.cfsec_rs_split(e._h, data.ctypes.data, length, cap, out, None, 0, ctypes.byref(need))
    per = (length + k - 1) // k
    each = (per + 63) // 64 * 64
    full = min(min(cap, per * tot) // per, tot) if cap > length else min(length // per, tot)
    npad = tot - full
    if npad == 0:
        assert st == 0 and need.value == 0
    else:
        assert st == _lib.ErrInvalidArg.status and need.value == npad * each + 63
        for shift in range(3):  # any start: the engine aligns inside the buffer
            raw = np.zeros(need.value + 64, np.uint8)
            pad_ptr = raw.ctypes.data + shift
            st = L.cfsec_rs_split(e._h, data.ctypes.data, length, cap, out, pad_ptr, need.value, ctypes.byref(need))
            assert st == 0
            base = out[full].data
            assert base % 64 == 0 and 0 <= base - pad_ptr < 64
            for j in range(npad):
                assert out[full + j].data == base + j * each and out[full + j].len == per
                assert out[full + j].cap == each
    for i in range(full):
        assert out[i].data == data.ctypes.data + i * per and out[i].len == per and out[i].cap == per
    got = [bytes(ctypes.string_at(out[i].data, per)) for i in range(tot)]
    assert got == py_split(k, tot, ref, length)


@pytest.mark.parametrize("k,m", [(6, 6), (12, 4), (15, 12), (1, 1)])
@pytest.mark.parametrize("length,cap", [(1, 1), (11, 11), (11, 1024), (1000, 1000), (1000, 1003), (4096, 8192)])
def test_split_join(k, m, length, cap):
    from chubaofs_amd import reedsolomon
    e = reedsolomon.New(k, m)
    r = np.random.default_rng(length)
    data = r.integers(0, 256, cap, dtype=np.uint8)
    ref = data.copy()
    shards = e.Split(data, length)
    assert len(shards) == k + m
    want = py_split(k, k + m, ref, length)
    assert [bytes(s) for s in shards] == want
    buf = io.BytesIO()
    e.Join(buf, shards, length)
    assert buf.getvalue() == ref[:length].tobytes()


def test_split_join_errors():
    from chubaofs_amd import reedsolomon
    e = reedsolomon.New(4, 2)
    with pytest.raises(_lib.ErrShortData):
        e.Split(np.zeros(0, np.uint8))
    sh = e.Split(np.arange(20, dtype=np.uint8))
    with pytest.raises(_lib.ErrShortData):
        e.Join(io.BytesIO(), sh, 1000)
    with pytest.raises(_lib.ErrTooFewShards):
        e.Join(io.BytesIO(), sh[:3], 10)
    sh2 = list(sh)
    sh2[0] = None
    with pytest.raises(_lib.ErrReconstructRequired):
        e.Join(io.BytesIO(), sh2, 10)


def test_codemode_table_c_matches_python():
    L = _lib.lib()
    for mode in list(cm._TACTICS):
        t = _lib.TacticC()
        assert L.cfsec_codemode_tactic(mode, ctypes.byref(t)) == 0
        p = cm.GetTactic(mode)
        assert (t.n, t.m, t.l, t.az_count, t.put_quorum, t.get_quorum, t.min_shard_size) == \
               (p.N, p.M, p.L, p.AZCount, p.PutQuorum, p.GetQuorum, p.MinShardSize)
    assert L.cfsec_codemode_tactic(99, ctypes.byref(_lib.TacticC())) == _lib.ErrInvalidCodeMode.status


def test_new_encoder_invalid_codemode():
    """encoder_test.go:40-51"""
    from chubaofs_amd import ec
    with pytest.raises(_lib.ErrInvalidCodeMode):
        ec.NewEncoder(ec.Config(CodeMode=cm.Tactic()))
    ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC15P12)))
    ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC16P20L2)))


def test_shards_in_idc_index_maps():
    from chubaofs_amd import ec
    e = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC6P10L2)))
    assert e.shards_in_idc(0) == [0, 1, 2, 6, 7, 8, 9, 10, 16]
    assert e.shards_in_idc(1) == [3, 4, 5, 11, 12, 13, 14, 15, 17]
    assert e.shards_in_idc(2) == []
    e2 = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC15P12)))
    assert e2.shards_in_idc(1) == [5, 6, 7, 8, 9, 19, 20, 21, 22]


def test_lrc_encode_invalid_shards():
    """encoder_test.go:126-128: wrong shard count -> ErrInvalidShards before any device use."""
    from chubaofs_amd import ec
    e = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC6P10L2), EnableVerify=True))
    shards = e.Split(np.frombuffer(b"Hello world", np.uint8).copy())
    assert len(shards) == 18
    with pytest.raises(_lib.ErrInvalidShards):
        e.Encode(shards[:-1])
    with pytest.raises(_lib.ErrInvalidShards):
        e.Encode([])


def test_get_shards_helpers():
    from chubaofs_amd import ec
    e = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC6P10L2)))
    shards = e.Split(np.frombuffer(b"Hello world", np.uint8).copy())
    assert len(e.GetDataShards(shards)) == 6
    assert len(e.GetParityShards(shards)) == 10
    assert len(e.GetLocalShards(shards)) == 2
    assert len(e.GetShardsInIdc(shards, 0)) == 9
    e2 = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC15P12)))
    s2 = e2.Split(np.frombuffer(b"Hello world", np.uint8).copy())
    assert e2.GetLocalShards(s2) == []
    assert len(e2.GetShardsInIdc(s2, 0)) == (15 + 12) // 3


def test_buffer_sizes():
    """buf_test.go:92-121"""
    from chubaofs_amd import ec
    kb, kb512 = 1024, 512 * 1024
    t = cm.GetTactic(cm.EC6P6)
    s = ec.GetBufferSizes(kb, t)
    shard = max((kb + t.N - 1) // t.N, t.MinShardSize)
    assert (s.ShardSize, s.DataSize, s.ECDataSize, s.ECSize) == (shard, kb, shard * t.N, shard * (t.N + t.M + t.L))
    t = cm.GetTactic(cm.EC16P20L2)
    s = ec.GetBufferSizes(kb512, t)
    shard = max((kb512 + t.N - 1) // t.N, t.MinShardSize)
    assert (s.ShardSize, s.ECSize) == (shard, shard * (t.N + t.M + t.L))
    for bad in (0, -1):
        with pytest.raises(_lib.ErrShortData):
            ec.GetBufferSizes(bad, t)
    # BASELINE shapes
    assert ec.GetBufferSizes(64 << 20, cm.GetTactic(cm.EC12P4)).ShardSize == 5592406
    assert ec.GetBufferSizes(4 << 20, cm.GetTactic(cm.EC12P4)).ShardSize == 349526
    assert ec.GetBufferSizes(1 << 20, cm.GetTactic(cm.EC6P6)).ShardSize == 174763
    assert ec.GetBufferSizes(4 << 20, cm.GetTactic(cm.EC6P10L2)).ShardSize == 699051
    assert ec.GetBufferSizes(4 << 20, cm.GetTactic(cm.EC16P20L2)).ShardSize == 262144
