"""The Scala 2.10.3 iteration-order restatements (product header gq_scala_order.h, compiled
for the host here; the oracle's scala_order) against the independent Python statement in
tests/scala_order_py.py.  Restated from the published Scala library, not observed on a JVM:
parity unpinned beyond this self-consistency and the Java String hash."""
import os
import subprocess

import numpy as np
import pytest

import scala_order_py as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_java_string_hash_known_values():
    # java.lang.String.hashCode, well known values
    assert S.java_string_hash("Seq") == 83007
    assert S.java_string_hash("") == 0
    assert S.java_string_hash("default") == (1544803905 & 0xFFFFFFFF)
    from guacamole_amd.soa import java_string_hash
    for s in ("default", "NA12878", "tumor", "s0", "é"):
        assert java_string_hash(s) == S.java_string_hash(s)


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    """tests/native/scala_order_check.cpp (gq_scala_order.h on the host) built with g++."""
    out = str(tmp_path_factory.mktemp("so") / "scala_order_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "guacamole_amd", "csrc"), "-o", out,
                           os.path.join(ROOT, "tests", "native", "scala_order_check.cpp")])
    return out


def test_product_header_matches_python(host_check):
    rng = np.random.default_rng(3)
    alleles = [("A", "C"), ("C", "C"), ("", ""), ("A", "ACGT"), ("GTT", "G"), ("N", "<ALT>")]
    alleles += [("".join(rng.choice(list("ACGTN"), rng.integers(0, 4))), "".join(rng.choice(list("ACGTN"),
                rng.integers(0, 4)))) for _ in range(40)]
    inp = "".join("%s %s\n" % (r or "-", a or "-") for r, a in alleles)
    out = subprocess.run([host_check], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    for (r, a), line in zip(alleles, out):
        h, bucket, trie = (int(x) for x in line.split())
        assert h == S.allele_hash(r, a)
        assert bucket == S.mutable_bucket(h)
        assert trie == S.trie_key(h)


def test_oracle_group_by_order_matches_python():
    from oracle import oracle as O
    rng = np.random.default_rng(4)
    for n in list(range(1, 20)) + [40, 100]:
        hashes = [int(x) for x in rng.integers(0, 2 ** 32, n, dtype=np.uint64)]
        assert O.scala_group_order(hashes) == S.group_by_order(hashes), n
    # colliding buckets keep the newest first; five keys switch to trie order
    assert O.scala_group_order([5, 5]) == S.group_by_order([5, 5])


def test_oracle_hashes_match_python():
    from oracle import oracle as O
    for r, a in (("A", "G"), ("C", "N"), ("", ""), ("AT", "A"), ("T", "TTG")):
        assert O.scala_allele_hash(r, a) == S.allele_hash(r, a)
    assert O.scala_genotype_hash(("A", "A"), ("A", "C")) == S.genotype_hash(("A", "A"), ("A", "C"))


def test_snv_bucket_table():
    """The single-base alleles (ref, b): every ref's five alleles fall in distinct buckets of the
    16-bucket table except (C, G) and (C, N) — the pair germline_proj sends to germline_complex."""
    collide = []
    for r in "ACGTN":
        bs = [S.mutable_bucket(S.allele_hash(r, b)) for b in "ACGTN"]
        for i in range(5):
            for j in range(i + 1, 5):
                if bs[i] == bs[j]:
                    collide.append((r, "ACGTN"[i], "ACGTN"[j]))
    assert collide == [("C", "G", "N")]
