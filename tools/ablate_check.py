"""Parity of the ablation arms (ablation build, OKV_ABLATE=1 with the arm's
knob set): the arm must be the path taken and its outputs equal the oracle's.
usage: OKV_ABLATE=1 <knob>=1 python tools/ablate_check.py stream|pieces|small_pieces|onepass
       OKV_ABLATE=1 python tools/ablate_check.py block|block512
       OKV_ABLATE=1 python tools/ablate_check.py enc_arms   (sets each encode knob itself)"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import objectkv_amd as okv  # noqa: E402
from objectkv_amd import _lib  # noqa: E402
from tests import test_decode_gpu as TD  # noqa: E402
from tests import test_encode_gpu as TE  # noqa: E402

arm = sys.argv[1]
assert _lib.LIB_PATH.endswith("libokv_sst_ablate.so"), _lib.LIB_PATH
if arm in ("stream", "small_pieces"):
    rng = np.random.default_rng(5)
    kinds = list(rng.choice(["s"] * 12 + ["M"], size=3000))
    seg, d = TD._mixed_segment(kinds, 8)
    dec = okv.Decoder(0)
    for index_only in (False, True):
        got = dec.decode(seg, d, index_only=index_only)
        if arm == "stream":
            assert dec.last_path() & _lib.PATH_STREAM, dec.last_path()
        TD._assert_same_as_oracle(got, seg, d, 0, index_only)
    dec.close()
elif arm == "pieces":
    n = 9000
    kinds = ["L"] * n
    for i in (0, 3, 1023, 1024, 1025, 4000, n - 1):
        kinds[i] = "M"
    seg, d = TD._mixed_segment(kinds, 21)
    seg = seg + bytes(4096)
    dec = okv.Decoder(0)
    for index_only in (False, True):
        got = dec.decode(seg, d, index_only=index_only)
        assert dec.last_path() & _lib.PATH_TILE, dec.last_path()
        TD._assert_same_as_oracle(got, seg, d, 0, index_only)
    dec.close()
elif arm == "onepass":
    enc = okv.Encoder(0)
    for T, vmax in ((50, 60), (3584, 120), (9000, 60), (3584, 3000)):
        rng = random.Random(T + vmax)
        rows = TE._random_rows(rng, 30000 if vmax <= 120 else 9000, 8, vmax)
        rc, want, meta = TE.oracle_segment(rows, T, 4096)
        got = enc.encode(rows, T, 4096, strict_go=rc == 0)
        if rc == 0:
            assert got.seg.tobytes() == want
        assert enc.last_path() & _lib.PATH_ENC_ONEPASS, enc.last_path()
    enc.close()
elif arm in ("block", "block512"):
    # OKV_VALUE_SWEEP=9 / 10 (set here): the one-launch per-block decode on
    # every large-block edge shape the tests use, against the oracle
    os.environ["OKV_VALUE_SWEEP"] = "9" if arm == "block" else "10"
    dec = okv.Decoder(0, flags=_lib.OPEN_NO_POINT)
    del os.environ["OKV_VALUE_SWEEP"]
    cases = []
    for seed in (1, 2):
        cases.append(TD._wide_segment(seed))
    rng = np.random.default_rng(11)
    cases.append(TD._mixed_segment(list(rng.choice(["s", "s", "L", "M"], size=300)), 5))
    for seed in (3, 4):
        cases.append(TD._tiny_value_segment(seed))
    w = okv.synth_segment(okv.sst.SYNTH_ZIPF, 7, nblocks=2000, threshold=57344, block_size=65536)
    cases.append((w.data().tobytes(), w.descs()[:2000]))
    # > kFastRows rows (the re-walk), a block over the 64 KiB stage (HBM walk)
    big = bytearray()
    for i in range(1500):
        big += (3).to_bytes(2, "little") + (5).to_bytes(4, "little") + b"k%02d" % (i % 100) + b"vvvvv"
    huge = bytearray()
    for i in range(30):
        huge += (8).to_bytes(2, "little") + (3000).to_bytes(4, "little") + b"K%07d" % i + bytes(3000)
    seg = bytes(big) + bytes(huge)
    d = np.array([(0, len(big), len(big), 0), (len(big), len(huge), len(huge), 0)], np.uint64)
    cases.append((seg, d))
    for seg, d in cases:
        n = max(1, d.shape[0])
        seg = bytes(seg) + bytes(max(0, 16385 * n - len(seg)) + 4096)  # large-block path
        got = dec.decode(seg, d)
        TD._assert_same_as_oracle(got, seg, d, 0, False)
    dec.close()
elif arm == "enc_arms":
    # the pack launch's variants that write whole segments (the others --
    # OKV_ENC_VARIANT 1, 2, 4, 5, 6 -- are diagnostics that skip work):
    # every one byte-equal to the oracle writer over many LDS regions
    enc = okv.Encoder(0)
    for knob, val in (("OKV_ENC_VARIANT", "8"), ("OKV_ENC_VARIANT", "9"),
                      ("OKV_ENC_VARIANT", "3"), ("OKV_ENC_IMAGE", "8192"),
                      ("OKV_ENC_IMAGE", "12288"), ("OKV_ENC_IMAGE", "32768"),
                      ("OKV_ENC_META_FUSED", "1")):
        os.environ[knob] = val
        for T, vmax in ((3584, 120), (3584, 60), (9000, 60)):
            rng = random.Random(T + vmax)
            rows = TE._random_rows(rng, 30000, 8, vmax)
            rc, want, meta = TE.oracle_segment(rows, T, 4096)
            got = enc.encode(rows, T, 4096, strict_go=rc == 0)
            if rc == 0:
                assert got.seg.tobytes() == want, (knob, val, T, vmax)
        del os.environ[knob]
        print(f"  {knob}={val}: parity ok", flush=True)
    enc.close()
print(f"ablation arm {arm}: parity ok")
