"""An independent Python statement of the Scala 2.10.3 iteration orders the reference's output
depends on (the C++ restatements: guacamole_amd/csrc/gq_scala_order.h for the product,
oracle/oracle.cpp scala_order for the checker).  Test helper: both are checked against it.

  MurmurHash3 (scala.util.hashing, 2.10): mix / mixLast / finalizeHash / productHash (seed
  0xcafebabe) / seqHash (seed "Seq".hashCode); mutable.HashTable: improve = byteswap32 rotated
  by the initial table's seed 4, bucket = the top log2(size) bits, chains prepend, iteration
  from the last bucket down; immutable.HashMap: improve(h) = h + ~(h << 9) ..., trie order by
  5-bit chunks from the lowest.
"""
M = 0xFFFFFFFF


def _rotl(x, r):
    x &= M
    return ((x << r) | (x >> (32 - r))) & M


def mix(h, k):
    k = (k * 0xcc9e2d51) & M
    k = _rotl(k, 15)
    k = (k * 0x1b873593) & M
    h ^= k
    h = _rotl(h, 13)
    return (h * 5 + 0xe6546b64) & M


def finalize_hash(h, n):
    h = (h ^ n) & M
    h ^= h >> 16
    h = (h * 0x85ebca6b) & M
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & M
    h ^= h >> 16
    return h


def java_string_hash(s: str) -> int:
    h = 0
    u = s.encode("utf-16-be")
    for i in range(0, len(u), 2):
        h = (31 * h + ((u[i] << 8) | u[i + 1])) & M
    return h


SEQ_SEED = java_string_hash("Seq")


def byte_seq_hash(bs: bytes) -> int:
    h = SEQ_SEED
    for b in bs:
        h = mix(h, (b - 256 if b >= 128 else b) & M)
    return finalize_hash(h, len(bs))


def allele_hash(ref: str, alt: str) -> int:
    return finalize_hash(mix(mix(0xcafebabe, byte_seq_hash(ref.encode("latin-1"))), byte_seq_hash(alt.encode("latin-1"))), 2)


def genotype_hash(a1, a2) -> int:
    seq = finalize_hash(mix(mix(SEQ_SEED, allele_hash(*a1)), allele_hash(*a2)), 2)
    return finalize_hash(mix(0xcafebabe, seq), 1)


def _byteswap32(v):
    hc = (v * 0x9e3775cd) & M
    hc = int.from_bytes(hc.to_bytes(4, "little"), "big")
    return (hc * 0x9e3775cd) & M


def mutable_bucket(h, bits=4):
    i = _byteswap32(h)
    improved = ((i >> 4) | (i << 28)) & M
    return (improved >> (32 - bits)) & ((1 << bits) - 1)


def trie_key(h):
    h = (h + (~(h << 9) & M)) & M
    h ^= h >> 14
    h = (h + (h << 4)) & M
    h ^= h >> 10
    k = 0
    for c in range(7):
        k = (k << 5) | ((h >> (5 * c)) & 31)
    return k


def group_by_order(hashes):
    """Positions of the keys (given in first-occurrence order) in groupBy's Map iteration order."""
    bits, table, n = 4, [[] for _ in range(16)], 0
    for i, h in enumerate(hashes):
        table[mutable_bucket(h, bits)].insert(0, i)
        n += 1
        if n > len(table) * 3 // 4:
            bits += 1
            nt = [[] for _ in range(2 * len(table))]
            for b in range(len(table) - 1, -1, -1):
                for e in table[b]:
                    nt[mutable_bucket(hashes[e], bits)].insert(0, e)
            table = nt
    order = [e for b in range(len(table) - 1, -1, -1) for e in table[b]]
    if len(order) > 4:
        order.sort(key=lambda e: trie_key(hashes[e]))  # stable: insertion order on equal keys
    return order
