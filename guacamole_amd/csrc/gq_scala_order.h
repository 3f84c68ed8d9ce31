// gq_scala_order.h — the iteration order of the Scala 2.10.3 collections the reference's
// output order depends on (host and device code of the library).  The oracle has its own,
// separate restatement (oracle/oracle.cpp scala_order), and the tests a third in Python
// (tests/scala_order_py.py): three independent statements checked against each other.
//
// Three sites of the reference iterate a hash-based collection and let that order reach the
// output (paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):
//   * commands/GermlineThresholdCaller.scala:103-104  elements.map(_.allele).groupBy(x => x)
//     .mapValues(_.length).toList ... sortBy(-count): a stable sort, so count ties keep the
//     groupBy map's order;
//   * pileup/Pileup.scala:57-61  bySample = elements.groupBy(sample name).map(...): the order
//     of the per-sample records at a locus (GermlineThresholdCaller.scala:100, .toSeq);
//   * commands/SomaticStandardCaller.scala:206-217  likelihoods.toMap.filter(...).map(_._2).sum:
//     the order the normal's variant-genotype likelihoods are added in.
// The algorithms restated here are the published Scala 2.10.3 library's (scala-library is a
// dependency absent from /root/reference, pom.xml:22):
//   * hash codes: case classes hash with MurmurHash3.productHash (seed 0xcafebabe, one mix per
//     field, finalizeHash(h, arity)); every Seq with MurmurHash3.seqHash (seed "Seq".hashCode,
//     one mix per element, finalizeHash(h, length)); a boxed Byte's ## is its (signed) value;
//     a String's ## is java.lang.String.hashCode.  Allele = (refBases, altBases)
//     (variants/Allele.scala:26), Genotype = (alleles: Allele*) (variants/Genotype.scala:38).
//   * TraversableLike.groupBy: a mutable.HashMap filled in element order, then an
//     immutable.Map built by iterating it.
//   * mutable.HashMap (HashTable): 16 buckets to start, load factor 0.75 (resize to twice the
//     size when more than 12 entries ... table.length * 3 / 4); bucket = the top log2(size)
//     bits of improve(hash, seed) = byteswap32(hash) rotated right by seed = bitCount(size - 1)
//     (the initial table's: seeds are not recomputed on resize); a new entry is prepended to
//     its bucket's chain; resize re-inserts old buckets from the last to the first, each chain
//     from its head.  Iteration: from the last populated bucket down to bucket 0, each chain
//     from its head.
//   * immutable.Map: up to four entries Map1..Map4 keep insertion order; from five on a
//     HashTrieMap whose iteration order is that of the 5-bit chunks of improve(hash) =
//     h + ~(h << 9); h ^ (h >>> 14); h + (h << 4); h ^ (h >>> 10), lowest chunk first
//     (a full 32-bit collision: a ListMap, insertion order).
// No JVM exists in this image, so these orders are restated, not observed: parity unpinned.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define GQ_HD __host__ __device__ __forceinline__
#else
#define GQ_HD inline
#endif

namespace gq {
namespace scala {

GQ_HD uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
GQ_HD uint32_t mix_last(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = rotl(k, 15);
  k *= 0x1b873593u;
  return h ^ k;
}
GQ_HD uint32_t mix(uint32_t h, uint32_t k) {
  h = mix_last(h, k);
  h = rotl(h, 13);
  return h * 5u + 0xe6546b64u;
}
GQ_HD uint32_t finalize_hash(uint32_t h, uint32_t n) {
  h ^= n;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
constexpr uint32_t kProductSeed = 0xcafebabeu;
constexpr uint32_t kSeqSeed = 83007u;  // "Seq".hashCode = 'S' * 31^2 + 'e' * 31 + 'q'

// Incremental MurmurHash3.seqHash over Byte elements (signed values).
struct SeqHasher {
  uint32_t h = kSeqSeed, n = 0;
  GQ_HD void add_byte(uint8_t b) {
    h = mix(h, (uint32_t)(int32_t)(int8_t)b);
    ++n;
  }
  GQ_HD void add_int(uint32_t v) {
    h = mix(h, v);
    ++n;
  }
  GQ_HD uint32_t result() const { return finalize_hash(h, n); }
};

// Allele(refBases, altBases).hashCode from the two Seq hashes
GQ_HD uint32_t allele_hash(uint32_t ref_seq_hash, uint32_t alt_seq_hash) {
  return finalize_hash(mix(mix(kProductSeed, ref_seq_hash), alt_seq_hash), 2);
}
// Genotype(a1, a2).hashCode: productHash over its one field, the Seq (a1, a2)
GQ_HD uint32_t genotype_hash(uint32_t a1, uint32_t a2) {
  SeqHasher s;
  s.add_int(a1);
  s.add_int(a2);
  return finalize_hash(mix(kProductSeed, s.result()), 1);
}
// java.lang.String.hashCode of Latin-1 bytes
GQ_HD uint32_t string_hash(const uint8_t *s, int n) {
  uint32_t h = 0;
  for (int i = 0; i < n; ++i) h = 31u * h + (uint32_t)s[i];
  return h;
}

// mutable.HashTable bucket of `hash` in a table of 2^bits buckets, with the seed of the
// initial 16-bucket table (4)
GQ_HD uint32_t byteswap32(uint32_t v) {
  uint32_t hc = v * 0x9e3775cdu;
  hc = (hc >> 24) | ((hc >> 8) & 0xFF00u) | ((hc << 8) & 0xFF0000u) | (hc << 24);
  return hc * 0x9e3775cdu;
}
GQ_HD uint32_t mutable_bucket(uint32_t hash, int bits, int seed = 4) {
  const uint32_t i = byteswap32(hash);
  const int rot = seed % 32;
  const uint32_t improved = rot ? ((i >> rot) | (i << (32 - rot))) : i;
  return (improved >> (32 - bits)) & ((1u << bits) - 1u);
}

// immutable.HashMap: the improved hash and its trie iteration key (the 5-bit chunks, lowest
// first, as the most significant digits); ascending keys = iteration order
GQ_HD uint32_t immutable_improve(uint32_t h) {
  h = h + ~(h << 9);
  h = h ^ (h >> 14);
  h = h + (h << 4);
  return h ^ (h >> 10);
}
GQ_HD uint64_t trie_key(uint32_t hash) {
  const uint32_t h = immutable_improve(hash);
  uint64_t k = 0;
  for (int c = 0; c < 7; ++c) k = (k << 5) | (uint64_t)((h >> (5 * c)) & 31u);
  return k;
}

}  // namespace scala
}  // namespace gq
