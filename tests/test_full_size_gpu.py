"""Full-size parity: the configurations the bench numbers are quoted on,
compared with the CPU oracle array for array at their real sizes -- the C3
segment (65 536 x 64 KiB, 4.30 GB), a larger C3-style segment (76 000 blocks)
whose block offsets and value arena pass 4 GiB, and the C4 encode of 100 M
rows (9.75 GB of blocks + the meta block of 2.38 M BlockStat entries).

Integer/byte work: every comparison is bit-exact.  Reference: the decode loop
segment_reader.go:338-352 (with :489-512), the writer segment_writer.go:80-328.
Host memory: ~15 GB (decode) / ~30 GB (encode); the GPU box allows 270 GiB."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import objectkv_amd as okv
from oracle import coracle as CO

pytestmark = pytest.mark.gpu

CHUNK = 1 << 28  # compare / copy 256 MiB at a time


def _same(a: np.ndarray, b: np.ndarray) -> bool:
    a, b = a.reshape(-1).view(np.uint8), b.reshape(-1).view(np.uint8)
    if a.size != b.size:
        return False
    return all(np.array_equal(a[i:i + CHUNK], b[i:i + CHUNK]) for i in range(0, a.size, CHUNK))


def _oracle_descs(d: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(d, np.uint64).view(CO.DESC_DTYPE).reshape(-1)


@pytest.mark.parametrize("nblk", [65536, 76000], ids=["c3_full_4.30GB", "c3_76k_arena_past_4GiB"])
def test_c3_full_decode_vs_oracle(decoder, nblk):
    """Every output array of the full decode (status, row_start, key/val
    bases, the SoA row index and both arenas) equals the oracle's."""
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 3, nblocks=nblk, threshold=57344,
                          block_size=65536)
    seg = w.data_view()
    d = w.descs()[:nblk]
    # C3's blocks end exactly at 4 GiB (its meta block lies past it); the
    # 76 000-block segment has block offsets and value-arena offsets past 4 GiB
    assert int(d[-1, 0] + d[-1, 1]) >= 1 << 32 and seg.nbytes > 1 << 32
    got = decoder.decode(seg, d)
    ref = CO.decode_soa(seg, _oracle_descs(d))
    assert int(got.status.max()) == 0
    for k in ("status", "row_start", "key_base", "val_base", "key_off", "key_len", "val_off",
              "val_len"):
        assert _same(getattr(got, k), ref[k]), k
    assert _same(got.key_arena, ref["key_arena"]), "key_arena"
    assert _same(got.val_arena, ref["val_arena"]), "val_arena"
    if nblk == 76000:
        assert int(d[-1, 0]) > 1 << 32
        assert got.val_arena.size > 1 << 32 and int(got.val_off[-1]) > 1 << 32


def test_c4_full_encode_vs_oracle():
    """The 100 M-row C4 encode (16 B keys, 64 B values, 3584 / 4096): the whole
    segment file -- 2 380 953 data blocks, the meta block with every
    BlockStat (offset, sizes, XXH64 hash) and the trailer -- equals the oracle
    writer's bytes."""
    n, kl, vl = 100_000_000, 16, 64
    enc = okv.Encoder(0)
    dev = torch.device("cuda", 0)
    t = dict(key_arena=torch.empty(n * kl, dtype=torch.uint8, device=dev),
             key_off=torch.empty(n, dtype=torch.int64, device=dev),
             key_len=torch.empty(n, dtype=torch.int16, device=dev),
             val_arena=torch.empty(n * vl, dtype=torch.uint8, device=dev),
             val_off=torch.empty(n, dtype=torch.int64, device=dev),
             val_len=torch.empty(n, dtype=torch.int32, device=dev))
    enc.synth_fixed_device(1, 0, n, kl, vl, t)
    nb = -(-n // 42)
    seg_t = torch.empty(nb * 4096 + (nb + 1) * (42 + kl) + 4096, dtype=torch.uint8, device=dev)
    eo = enc.encode_device(t, n, {"seg": seg_t}, strict_go=True)
    assert eo.n_blocks == nb == 2_380_953 and eo.data_bytes == nb * 4096
    host = {k: v.cpu().numpy() for k, v in t.items()}
    del t
    for k, dt in (("key_off", np.uint64), ("val_off", np.uint64), ("key_len", np.uint16),
                  ("val_len", np.uint32)):
        host[k] = host[k].view(dt)
    want = CO.encode_soa(host, n, 3584, 4096)
    assert want.rc == 0 and eo.file_bytes == want.file.size
    for i in range(0, want.file.size, CHUNK):
        j = min(want.file.size, i + CHUNK)
        assert np.array_equal(seg_t[i:j].cpu().numpy(), want.file[i:j]), f"bytes {i}..{j}"
    enc.close()


# ---- every rank's workload of the multi-GPU configs, on one GPU ---------------
# (bench.py CONFIGS: C5 rank k decodes its own 16 384-block segment of seed 3 + k;
# C4 at N GPUs encodes rows [100 M k / N, 100 M (k + 1) / N) of seed 1 as one segment)

@pytest.mark.parametrize("rank", range(1, 8))
def test_c5_rank_segment_vs_oracle(decoder, rank):
    """C5 rank k's 1 GiB segment (16 384 x 64 KiB, seed 3 + k): every output
    array equals the oracle's (rank 0's is the C3 prefix, covered above)."""
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 3 + rank, nblocks=16384, threshold=57344,
                          block_size=65536)
    seg = w.data_view()
    d = w.descs()[:16384]
    got = decoder.decode(seg, d)
    ref = CO.decode_soa(seg, _oracle_descs(d))
    assert int(got.status.max()) == 0
    for k in ("status", "row_start", "key_base", "val_base", "key_off", "key_len", "val_off",
              "val_len"):
        assert _same(getattr(got, k), ref[k]), k
    assert _same(got.key_arena, ref["key_arena"]), "key_arena"
    assert _same(got.val_arena, ref["val_arena"]), "val_arena"


@pytest.mark.parametrize("rank", [1, 7])
def test_c4_key_range_shard_vs_oracle(rank):
    """C4 at 8 GPUs: rank k's key-range shard (rows 12.5 M k .. 12.5 M (k + 1) - 1,
    i.e. 87.5 M .. 99 999 999 for the last) encoded as its own segment: the
    whole file equals the oracle writer's over the same rows."""
    total, world, kl, vl = 100_000_000, 8, 16, 64
    lo, hi = total * rank // world, total * (rank + 1) // world
    n = hi - lo
    enc = okv.Encoder(0)
    dev = torch.device("cuda", 0)
    t = dict(key_arena=torch.empty(n * kl, dtype=torch.uint8, device=dev),
             key_off=torch.empty(n, dtype=torch.int64, device=dev),
             key_len=torch.empty(n, dtype=torch.int16, device=dev),
             val_arena=torch.empty(n * vl, dtype=torch.uint8, device=dev),
             val_off=torch.empty(n, dtype=torch.int64, device=dev),
             val_len=torch.empty(n, dtype=torch.int32, device=dev))
    enc.synth_fixed_device(1, lo, n, kl, vl, t)
    nb = -(-n // 42)
    seg_t = torch.empty(nb * 4096 + (nb + 1) * (42 + kl) + 4096, dtype=torch.uint8, device=dev)
    eo = enc.encode_device(t, n, {"seg": seg_t}, strict_go=True)
    assert eo.n_blocks == nb and eo.data_bytes == nb * 4096
    host = {k: v.cpu().numpy() for k, v in t.items()}
    del t
    for k, dt in (("key_off", np.uint64), ("val_off", np.uint64), ("key_len", np.uint16),
                  ("val_len", np.uint32)):
        host[k] = host[k].view(dt)
    # the shard's first key is row lo's big-endian index
    assert host["key_arena"][:kl].tobytes() == lo.to_bytes(kl, "big")
    want = CO.encode_soa(host, n, 3584, 4096)
    assert want.rc == 0 and eo.file_bytes == want.file.size
    for i in range(0, want.file.size, CHUNK):
        j = min(want.file.size, i + CHUNK)
        assert np.array_equal(seg_t[i:j].cpu().numpy(), want.file[i:j]), f"bytes {i}..{j}"
    enc.close()
