"""CPU: the host code that parses untrusted bytes, under AddressSanitizer + UndefinedBehaviorSanitizer.

SURVEY §5 asks for ASan/UBSan builds of the host C++; the reference guards the same ground with
miri and a libfuzzer target (.github/workflows/ci.yml:58-72, fuzz/src/lib.rs:56-150).  Two
harnesses (tests/fuzz/, built by `make -C vortex_amd/csrc sanitize` with
-fsanitize=address,undefined -fno-sanitize-recover=all; host code only, no HIP):

* vxfile_fuzz -- seeded mutations (bit flips, boundary words, truncations, insertions,
  deletions, block copies; half aimed at the footer and the chunks' message headers) of small
  Vortex files written by tools/vxfile.py: the lineitem table and one file per encoding.  Every
  mutated file must give InvalidSerde / NotImplemented (an encoding id nobody registered, as the
  reference's registry answers) or trees whose every buffer lies inside the file
  (vortex-serde/src/message_reader.rs:249-348 restated by vortex_amd/csrc/serde.cpp).
* codec_san -- the encoders (encode.cpp) and the oracle round-trip seeded random inputs of every
  ptype, length and edge value; the oracle's parsers of untrusted bytes are fed garbage.

A sanitizer report aborts the harness (non-zero exit), so the tests fail on any finding.
"""
import json
import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "vortex_amd" / "csrc"
SAN = CSRC / "build_san"


@pytest.fixture(scope="module")
def harnesses():
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    r = subprocess.run(["make", "-C", str(CSRC), "sanitize"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return SAN


def _run(cmd, timeout=600):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        f"rc={r.returncode}\n{r.stderr[-4000:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


def _seed_files(tmp_path):
    from tools import lineitem as LI
    from tools import vxfile as X
    import vortex_amd.arrays as A
    import vortex_amd.encode as E
    cols, _ = LI.lineitem_columns(range(LI.n_chunks(3000, 1024)), rows=3000, chunk_rows=1024)
    written = []
    for name, _ in LI.COLUMNS:
        chunks = cols[name].children[1:]
        if name in LI.DATE_COLUMNS:
            chunks = [X.date_column(c) for c in chunks]
        written.append((name, chunks))
    seeds = [("lineitem", X.write_file(written))]
    rng = np.random.default_rng(5)
    n = 1500
    arrays = {
        "delta": E.encode_delta(np.cumsum(rng.integers(0, 9, n)).astype(np.uint32)),
        "zigzag": E.encode_zigzag(rng.integers(-500, 500, n).astype(np.int32)),
        "alprd": E.encode_alprd(rng.standard_normal(n)),
        "alp_patched": E.encode_alp(np.concatenate([np.round(rng.uniform(0, 100, n - 3), 2), [np.pi, np.e, 1e300]])),
        "bitpacked_patched": E.encode_bitpacked(np.where(rng.random(n) < 0.01, 1 << 40,
                                                         rng.integers(0, 100, n)).astype(np.uint64)),
        "runend": E.encode_runend(np.repeat(rng.integers(0, 50, 150), 10).astype(np.int64), compress_values=True),
        "dict_strings": E.encode_dict_strings([b"mode-%d" % (i % 7) for i in range(n)]),
        "fsst": E.encode_fsst([None if i % 17 == 0 else b"hello world %d" % i for i in range(n)]),
        "varbinview": E.encode_varbinview([None if i % 5 == 0 else b"x" * (i % 30) for i in range(n)]),
        "bool": A.bool_array(rng.random(n) < 0.5, validity=rng.random(n) < 0.9, bit_offset=3),
        "runend_bool": E.encode_runend_bool(np.repeat(rng.random(15) < 0.5, 100), bitpack_ends=True),
        "roaring_validity": A.primitive(rng.integers(0, 9, n).astype(np.int16),
                                        validity=E.encode_roaring_bool(rng.random(n) < 0.9)),
        "sparse": A.sparse(A.primitive(np.array([3, 70, 999], np.uint64)), A.primitive(np.array([1, 2, 3], np.int32)),
                           1000, fill=-7),
        "constant": A.constant(-2.25, 500, "f32"),
    }
    for name, a in arrays.items():
        seeds.append((name, X.write_file([(name, [a])])))
    paths = []
    for name, data in seeds:
        p = tmp_path / f"{name}.vortex"
        p.write_bytes(data)
        paths.append(p)
    return paths


def test_file_reader_mutation_fuzz(harnesses, tmp_path):
    """>= 10,000 seeded mutations; InvalidSerde / NotImplemented or in-file trees, nothing else."""
    paths = _seed_files(tmp_path)
    total = opened = trees = 0
    statuses: dict = {}
    for i, p in enumerate(paths):
        iters = 4000 if i == 0 else 500
        r = _run([harnesses / "vxfile_fuzz", p, iters, 1000 + i])
        assert r["bad_trees"] == 0, (p.name, r)
        total += r["iterations"]
        opened += r["opened"]
        trees += r["trees"]
        for k, v in r["status"].items():
            statuses[int(k)] = statuses.get(int(k), 0) + v
    assert total >= 10_000
    assert opened > 0 and trees > 0  # some mutations leave a parseable file: its trees were checked
    assert set(statuses) <= {4, 5}, statuses  # InvalidSerde, NotImplemented (unknown encoding id)


def test_encoders_and_oracle_under_sanitizers(harnesses):
    r = _run([harnesses / "codec_san", 2500, 11])
    assert r["failures"] == 0 and r["iterations"] == 2500
