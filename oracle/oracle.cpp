/*
 * oracle.cpp — CPU restatement of Guacamole's pileup + per-locus caller path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  The product (guacamole_amd/) never
 * links or calls this file; it is the checker for tests/, smoke() and the
 * bench's cpu_baseline leg.
 *
 * Every block below cites the reference file:line it restates.  Paths are
 * relative to /root/reference/src/main/scala/org/hammerlab/guacamole/.
 *
 * Parity pinning: the KATs transcribed in tests/test_oracle_kats.py (PileupSuite,
 * GermlineThresholdCallerSuite, SomaticStandardCallerSuite, LikelihoodSuite,
 * AlleleEvidenceSuite, MDTagUtilsSuite, DistributedUtilSuite) run against this
 * file.  Third-party behaviour restated from the published algorithms (not in
 * /root/reference): ADAM 0.18.1 MdTag / PhredUtils, htsjdk 1.118 CigarOperator,
 * Colt 1.2.0 DoubleMatrix1D.aggregate (folds last->first), Scala 2.10
 * mutable.PriorityQueue (heap array order), Breeze 0.11 mean/median, java.lang.StrictMath
 * log / exp / log10 (fdlibm 5.3, strictmath.h).
 */
#include "oracle.h"
#include "strictmath.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <functional>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string g_err;

struct OracleError : std::runtime_error {
  int code;
  OracleError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
enum { E_ASSERT = 1, E_INVALID_CIGAR = 2, E_MD = 3, E_NO_MD = 4, E_MULTI_REF = 5, E_UNSORTED = 6, E_ARG = 7 };

[[noreturn]] void fail(int code, const std::string &m) { throw OracleError(code, m); }

// htsjdk CigarOperator (BAM op codes) -------------------------------------------------
enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };
inline bool consumesRead(int op) { return op == OP_M || op == OP_I || op == OP_S || op == OP_EQ || op == OP_X; }
inline bool consumesRef(int op) { return op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X; }

struct CigarEl {
  int op;
  int len;
};
// CigarUtils.scala:30-42
inline int cigarReadLength(const CigarEl &c) { return consumesRead(c.op) ? c.len : 0; }
inline int cigarRefLength(const CigarEl &c) { return consumesRef(c.op) ? c.len : 0; }

inline bool isStandardBase(uint8_t b) { return b == 'A' || b == 'C' || b == 'G' || b == 'T'; }  // Bases.scala:67-69

// ADAM MdTag(mdTag, referenceStart, cigar) restated: MD letters/runs are mapped to
// the reference positions consumed by M/=/X/D cigar ops, N gaps skipped (pinned by
// MDTagUtilsSuite "RNA read with N CIGAR operator").  Digits = matches, letters =
// mismatches (reference base), '^' + letters = deleted reference bases.
struct MdTag {
  std::unordered_map<int64_t, uint8_t> mismatches, deletions;
  int64_t start = 0;
  int countOfMismatches() const { return (int)mismatches.size(); }
};

struct MdCursor {  // k-th MD-consumed position -> reference position
  const std::vector<CigarEl> &cig;
  size_t ci = 0;
  int within = 0;
  int64_t rp;
  int64_t last;
  bool exhausted = false;
  MdCursor(const std::vector<CigarEl> &c, int64_t start) : cig(c), rp(start), last(start - 1) {}
  int64_t next() {
    while (ci < cig.size()) {
      const CigarEl &c = cig[ci];
      bool mdConsumed = c.op == OP_M || c.op == OP_EQ || c.op == OP_X || c.op == OP_D;
      if (mdConsumed && within < c.len) {
        int64_t p = rp + within;
        ++within;
        last = p;
        return p;
      }
      rp += cigarRefLength(c);
      ++ci;
      within = 0;
    }
    return ++last;  // MD longer than the alignment: keep counting linearly (plain MdTag)
  }
  void skip(int64_t n) {
    for (int64_t i = 0; i < n; ++i) next();
  }
};

MdTag parseMdTag(const char *s, int len, int64_t refStart, const std::vector<CigarEl> &cig) {
  MdTag t;
  t.start = refStart;
  MdCursor cur(cig, refStart);
  int off = 0;
  auto up = [](char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; };
  auto isAlpha = [&](char c) { c = up(c); return c >= 'A' && c <= 'Z'; };
  auto readMatches = [&]() {
    if (off >= len || !(s[off] >= '0' && s[off] <= '9'))
      fail(E_MD, "MdTag " + std::string(s, len) + " does not have a digit where one is required");
    int64_t n = 0;
    while (off < len && s[off] >= '0' && s[off] <= '9') n = n * 10 + (s[off++] - '0');
    cur.skip(n);
  };
  if (len <= 0) return t;
  readMatches();
  while (off < len) {
    if (s[off] == '^') {
      ++off;
      while (off < len && isAlpha(s[off])) t.deletions[cur.next()] = (uint8_t)up(s[off++]);
    } else if (isAlpha(s[off])) {
      while (off < len && isAlpha(s[off])) t.mismatches[cur.next()] = (uint8_t)up(s[off++]);
    } else {
      fail(E_MD, "Invalid MdTag character in " + std::string(s, len));
    }
    readMatches();
  }
  return t;
}

// reads/MappedRead.scala:35-111 -----------------------------------------------------------
struct Read {
  int64_t index;
  int32_t contig;
  int64_t start, end;
  int mapq;
  bool positive;
  int sample;
  std::string sampleName;  // Option(read.sampleName).getOrElse("default") (Pileup.scala:58)
  const uint8_t *seq;
  const uint8_t *qual;
  int len;
  std::vector<CigarEl> cigar;
  bool hasMd = false;
  MdTag md;
  mutable std::vector<uint8_t> mdRef;
  mutable bool mdRefBuilt = false;

  bool overlapsLocus(int64_t l) const { return start <= l && l < end; }  // HasReferenceRegion.scala:51-53

  // MDTagUtils.getReference (MDTagUtils.scala:23-78), allowNBase = true (MappedRead.scala:57-65)
  const std::vector<uint8_t> &mdTagReferenceBases() const {
    if (mdRefBuilt) return mdRef;
    if (!hasMd) fail(E_NO_MD, "Attempted to get reference data for a read without an MD tag");
    int64_t refPos = md.start;
    int readPos = 0;
    std::vector<uint8_t> ref;
    ref.reserve((size_t)std::max<int64_t>(0, end - start));
    for (const CigarEl &c : cigar) {
      if (c.op == OP_M || c.op == OP_EQ || c.op == OP_X) {
        for (int i = 0; i < c.len; ++i) {
          auto it = md.mismatches.find(refPos);
          if (it != md.mismatches.end()) ref.push_back(it->second);
          else {
            if (readPos >= len) fail(E_ASSERT, "read sequence shorter than CIGAR");
            ref.push_back(seq[readPos]);
          }
          ++readPos;
          ++refPos;
        }
      } else if (c.op == OP_N) {
        refPos += c.len;
        ref.insert(ref.end(), (size_t)c.len, (uint8_t)'N');
      } else if (c.op == OP_D) {
        for (int i = 0; i < c.len; ++i) {
          auto it = md.deletions.find(refPos);
          if (it == md.deletions.end())
            fail(E_MD, "Cigar seems inconsistent with MD tag: could not find deleted base");
          ref.push_back(it->second);
          ++refPos;
        }
      } else {
        if (consumesRead(c.op)) readPos += c.len;
        if (consumesRef(c.op)) fail(E_MD, "Cannot handle operator");
      }
    }
    mdRef.swap(ref);
    mdRefBuilt = true;
    return mdRef;
  }
  // MappedRead.getReferenceBaseAtLocus (MappedRead.scala:69-76)
  uint8_t referenceBaseAtLocus(int64_t l) const {
    if (!(l >= start && l < end)) fail(E_ASSERT, "assumption failed: locus outside read");
    const auto &r = mdTagReferenceBases();
    int64_t i = l - start;
    if (i < 0 || i >= (int64_t)r.size()) fail(E_ASSERT, "reference index out of bounds");
    return r[(size_t)i];
  }
  // PhredUtils.phredToSuccessProbability(alignmentQuality)  (MappedRead.scala:78)
  double alignmentLikelihood() const;
};

// ADAM PhredUtils restated
double phredToErrorProbability(int phred) {
  if (phred > 255) phred = 255;
  if (phred < 0) fail(E_ASSERT, "negative phred");
  return std::pow(10.0, -phred / 10.0);
}
double phredToSuccessProbability(int phred) { return 1.0 - phredToErrorProbability(phred); }
int probabilityToPhred(double p) {
  double x = -10.0 * strictmath::log10(p);
  // java Math.round(double) = floor(x + 0.5), saturating; .toInt truncates the long
  if (std::isnan(x)) return 0;
  double r = std::floor(x + 0.5);
  long long l;
  if (r >= 9.2233720368547758e18) l = INT64_MAX;
  else if (r <= -9.2233720368547758e18) l = INT64_MIN;
  else l = (long long)r;
  return (int)(int32_t)(uint32_t)(uint64_t)l;
}
int successProbabilityToPhred(double p) { return probabilityToPhred(1.0 - p); }
double Read::alignmentLikelihood() const { return phredToSuccessProbability(mapq); }

// variants/Allele.scala:26-43 --------------------------------------------------------------
struct Allele {
  std::string ref, alt;
  bool isVariant() const { return ref != alt; }
  bool operator==(const Allele &o) const { return ref == o.ref && alt == o.alt; }
  bool operator<(const Allele &o) const {  // BasesOrdering: string compare ref then alt
    int c = ref.compare(o.ref);
    if (c != 0) return c < 0;
    return alt.compare(o.alt) < 0;
  }
};
struct AlleleHash {
  size_t operator()(const Allele &a) const { return std::hash<std::string>()(a.ref) * 1000003u ^ std::hash<std::string>()(a.alt); }
};

// ---- Scala 2.10.3 hash-collection iteration order (scala-library 2.10.3, pom.xml:22;
// restated from its published sources: MurmurHash3, mutable.HashTable, immutable.HashMap,
// TraversableLike.groupBy).  Parity unpinned: no JVM here to observe it.
namespace scala_order {
uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
uint32_t mix(uint32_t h, uint32_t k) {  // MurmurHash3.mix
  k *= 0xcc9e2d51u;
  k = rotl(k, 15);
  k *= 0x1b873593u;
  h ^= k;
  h = rotl(h, 13);
  return h * 5u + 0xe6546b64u;
}
uint32_t finalizeHash(uint32_t h, uint32_t len) {  // MurmurHash3.finalizeHash (avalanche(h ^ len))
  h ^= len;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
uint32_t javaStringHash(const std::string &s) {  // java.lang.String.hashCode
  uint32_t h = 0;
  for (unsigned char c : s) h = 31u * h + c;
  return h;
}
const uint32_t kSeqSeed = javaStringHash("Seq"), kProductSeed = 0xcafebabeu;
uint32_t byteSeqHash(const std::string &bytes) {  // MurmurHash3.seqHash of a Seq[Byte] (## = signed value)
  uint32_t h = kSeqSeed;
  for (unsigned char c : bytes) h = mix(h, (uint32_t)(int32_t)(int8_t)c);
  return finalizeHash(h, (uint32_t)bytes.size());
}
uint32_t alleleHash(const Allele &a) {  // case class Allele(refBases, altBases): productHash
  return finalizeHash(mix(mix(kProductSeed, byteSeqHash(a.ref)), byteSeqHash(a.alt)), 2);
}
uint32_t genotypeHash(const Allele &a1, const Allele &a2) {  // case class Genotype(alleles: Allele*)
  const uint32_t seq = finalizeHash(mix(mix(kSeqSeed, alleleHash(a1)), alleleHash(a2)), 2);
  return finalizeHash(mix(kProductSeed, seq), 1);
}
// mutable.HashTable.index: the top log2(size) bits of improve(hash, seed), improve =
// byteswap32(hash) rotated right by seed (the initial 16-bucket table's bitCount(15) = 4)
uint32_t mutableIndex(uint32_t hash, int bits) {
  uint32_t hc = hash * 0x9e3775cdu;
  hc = (hc >> 24) | ((hc >> 8) & 0xFF00u) | ((hc << 8) & 0xFF0000u) | (hc << 24);
  const uint32_t i = hc * 0x9e3775cdu;
  const uint32_t improved = (i >> 4) | (i << 28);
  return (improved >> (32 - bits)) & ((1u << bits) - 1u);
}
// immutable.HashMap.improve, and the HashTrieMap iteration key: 5-bit chunks, lowest first
uint64_t trieKey(uint32_t h) {
  h = h + ~(h << 9);
  h = h ^ (h >> 14);
  h = h + (h << 4);
  h = h ^ (h >> 10);
  uint64_t k = 0;
  for (int c = 0; c < 7; ++c) k = (k << 5) | (uint64_t)((h >> (5 * c)) & 31u);
  return k;
}
// Iteration order of the immutable Map groupBy returns for keys with these hashes, given in
// first-occurrence (insertion) order: positions into `hashes`.
//   mutable.HashMap filled in that order: 16 buckets, entry prepended to its chain, resize x2
//   when more than size * 3/4 entries (old buckets last to first, chains from the head);
//   iterated from the last populated bucket down, chains from the head;
//   immutable.Map built from that iteration: Map1..Map4 keep it; five or more keys form a
//   HashTrieMap (ascending trieKey; equal keys in insertion order, a ListMap).
std::vector<int> groupByOrder(const std::vector<uint32_t> &hashes) {
  int bits = 4;
  std::vector<std::vector<int>> table(16);
  size_t n = 0;
  for (int i = 0; i < (int)hashes.size(); ++i) {
    auto &chain = table[mutableIndex(hashes[(size_t)i], bits)];
    chain.insert(chain.begin(), i);
    if (++n > table.size() * 3 / 4) {
      std::vector<std::vector<int>> nt(table.size() * 2);
      ++bits;
      for (size_t b = table.size(); b-- > 0;)
        for (int e : table[b]) {
          auto &c2 = nt[mutableIndex(hashes[(size_t)e], bits)];
          c2.insert(c2.begin(), e);
        }
      table.swap(nt);
    }
  }
  std::vector<int> order;
  for (size_t b = table.size(); b-- > 0;)
    for (int e : table[b]) order.push_back(e);
  if (order.size() > 4)
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return trieKey(hashes[(size_t)a]) < trieKey(hashes[(size_t)b]); });
  return order;
}
}  // namespace scala_order

// pileup/Alignment.scala:32-94
enum Kind { K_MATCH, K_MISMATCH, K_INSERTION, K_DELETION, K_MIDDELETION, K_CLIPPED };
struct Evaluated {
  Kind kind;
  Allele allele;
  int quality;
};

// pileup/PileupElement.scala:40-274 ------------------------------------------------------------
struct Elem {
  const Read *read;
  int64_t locus;
  uint8_t referenceBase;
  int readPosition;
  int cigarElementIndex;
  int64_t cigarElementLocus;
  int indexWithinCigarElement;
  mutable bool evaluated = false;
  mutable Evaluated ev;

  const CigarEl &cigarElement() const {
    if (cigarElementIndex < 0 || cigarElementIndex >= (int)read->cigar.size())
      fail(E_ASSERT, "cigar element index out of bounds");
    return read->cigar[(size_t)cigarElementIndex];
  }
  bool currentCigarElementContainsLocus(int64_t l) const {  // :205-207
    const CigarEl &c = cigarElement();
    return cigarElementLocus <= l && l < cigarElementLocus + cigarRefLength(c);
  }
  Elem advanceToNextCigarElement() const {  // :176-198
    const CigarEl &c = cigarElement();
    int readPositionOffset = consumesRead(c.op) ? c.len - indexWithinCigarElement : 0;
    int64_t nextLocus = locus + (cigarRefLength(c) - indexWithinCigarElement);
    Elem e{read, nextLocus, (uint8_t)'N', readPosition + readPositionOffset, cigarElementIndex + 1,
           cigarElementLocus + cigarRefLength(c), 0, false, {}};
    return e;
  }
  Elem advanceToLocus(int64_t newLocus, uint8_t newReferenceBase) const {  // :220-248
    Elem e = *this;
    e.evaluated = false;
    for (;;) {
      if (!(newLocus >= e.locus)) fail(E_ASSERT, "Can't rewind; pileups only advance");
      if (!(newLocus < read->end)) fail(E_ASSERT, "This read stops before the requested locus");
      if (e.currentCigarElementContainsLocus(newLocus)) {
        const CigarEl &c = e.cigarElement();
        int rpo = consumesRead(c.op) ? (int)(newLocus - e.cigarElementLocus - e.indexWithinCigarElement) : 0;
        e.locus = newLocus;
        e.referenceBase = newReferenceBase;
        e.readPosition += rpo;
        e.indexWithinCigarElement = (int)(newLocus - e.cigarElementLocus);
        return e;
      } else if (newLocus == 0 && e.cigarElement().op == OP_I) {
        return e;
      } else {
        e = e.advanceToNextCigarElement();
      }
    }
  }
  static Elem create(const Read *read, int64_t locus, uint8_t referenceBase) {  // :264-274
    if (!(read->start < read->end)) fail(E_ASSERT, "assumption failed: locus < read.end");
    Elem e{read, read->start, (uint8_t)'N', 0, 0, read->start, 0, false, {}};
    return e.advanceToLocus(locus, referenceBase);
  }

  // :68-135 alignment, :157 allele, :166-171 qualityScore
  const Evaluated &evaluate() const {
    if (evaluated) return ev;
    const auto &cig = read->cigar;
    const CigarEl &c = cigarElement();
    bool isFinal = indexWithinCigarElement == c.len - 1;
    bool hasNext = cigarElementIndex + 1 < (int)cig.size();
    int nextOp = isFinal ? (hasNext ? cig[(size_t)cigarElementIndex + 1].op : -1) : c.op;
    auto makeInsertion = [&](const CigarEl &el) {
      int from = readPosition, until = readPosition + cigarReadLength(el) + 1;
      from = std::max(0, std::min(from, read->len));
      until = std::max(from, std::min(until, read->len));  // Seq.view slices clamp
      Evaluated r;
      r.kind = K_INSERTION;
      r.allele.alt.assign((const char *)read->seq + from, (size_t)(until - from));
      if (!r.allele.alt.empty()) r.allele.ref.assign(1, r.allele.alt[0]);
      if (until == from) fail(E_ASSERT, "empty insertion qualities (min of empty)");
      int q = 1 << 30;
      for (int i = from; i < until; ++i) q = std::min(q, (int)(int8_t)read->qual[i]);
      r.quality = q;
      return r;
    };
    Evaluated r;
    if ((c.op == OP_M || c.op == OP_EQ) && nextOp == OP_I) {
      r = makeInsertion(cig[(size_t)cigarElementIndex + 1]);
    } else if (c.op == OP_I && nextOp != -1 && cigarElementLocus == 0) {
      r = makeInsertion(c);
    } else if (c.op == OP_I) {
      fail(E_INVALID_CIGAR, "Should not have a PileupElement at non-reference-consuming cigar-operator I");
    } else if ((c.op == OP_M || c.op == OP_EQ || c.op == OP_X) && nextOp == OP_D) {
      if (!read->hasMd) fail(E_NO_MD, "None.get (mdTagOpt) for deletion");
      int64_t referenceStringIdx =
          (cigarElementLocus - read->start) + (consumesRef(c.op) ? indexWithinCigarElement : 0);
      int nlen = cig[(size_t)cigarElementIndex + 1].len;
      r.kind = K_DELETION;
      r.allele.ref.assign(1, (char)referenceBase);
      for (int64_t off = referenceStringIdx + 1; off < referenceStringIdx + 1 + nlen; ++off) {
        auto it = read->md.deletions.find(read->start + off);
        if (it == read->md.deletions.end()) fail(E_MD, "key not found in MdTag deletions");
        r.allele.ref.push_back((char)it->second);
      }
      r.allele.alt.assign(1, (char)referenceBase);
      r.quality = (int)(int8_t)read->qual[readPosition];
    } else if (c.op == OP_D) {
      if (!read->hasMd) fail(E_NO_MD, "None.get (mdTagOpt) for mid-deletion");
      auto it = read->md.deletions.find(locus);
      if (it == read->md.deletions.end()) fail(E_MD, "key not found in MdTag deletions");
      r.kind = K_MIDDELETION;
      r.allele.ref.assign(1, (char)it->second);
      r.quality = read->mapq;
    } else if (nextOp == OP_D) {
      fail(E_ASSERT, "Found deletion preceded by unexpected cigar operator");
    } else if (c.op == OP_M || c.op == OP_EQ || c.op == OP_X) {
      if (readPosition < 0 || readPosition >= read->len) fail(E_ASSERT, "read position out of bounds");
      uint8_t base = read->seq[readPosition];
      r.kind = base == referenceBase ? K_MATCH : K_MISMATCH;
      r.allele.ref.assign(1, (char)referenceBase);
      r.allele.alt.assign(1, (char)base);
      r.quality = (int)(int8_t)read->qual[readPosition];
    } else if (c.op == OP_S || c.op == OP_N || c.op == OP_H) {
      r.kind = K_CLIPPED;
      r.quality = read->mapq;
    } else {
      fail(E_ASSERT, "`P` CIGAR-ops should have been ignored earlier");
    }
    ev = r;
    evaluated = true;
    return ev;
  }
};

// Scala 2.10 collection.mutable.PriorityQueue (heap array, index 0 unused) with the
// SlidingWindow ordering "compare(a, b) = b.end compare a.end" (SlidingWindow.scala:62-68).
struct ScalaPQ {
  std::vector<const Read *> a{nullptr};
  static bool lt(const Read *x, const Read *y) { return y->end < x->end; }
  static bool gteq(const Read *x, const Read *y) { return y->end >= x->end; }
  bool empty() const { return a.size() < 2; }
  const Read *head() const { return a[1]; }
  void fixUp(size_t k) {
    while (k > 1 && lt(a[k / 2], a[k])) {
      std::swap(a[k], a[k / 2]);
      k /= 2;
    }
  }
  void fixDown(size_t m, size_t n) {
    size_t k = m;
    while (n >= 2 * k) {
      size_t j = 2 * k;
      if (j < n && lt(a[j], a[j + 1])) ++j;
      if (gteq(a[k], a[j])) return;
      std::swap(a[k], a[j]);
      k = j;
    }
  }
  void enqueue(const Read *r) {
    a.push_back(r);
    fixUp(a.size() - 1);
  }
  const Read *dequeue() {
    size_t size0 = a.size() - 1;  // new p_size0
    std::swap(a[1], a[size0]);
    fixDown(1, size0 - 1);
    const Read *r = a[size0];
    a.pop_back();
    return r;
  }
};

// windowing/SlidingWindow.scala:45-128 (halfWindowSize = 0)
struct Window {
  std::vector<const Read *> sorted;
  size_t next = 0;
  int64_t currentLocus = -1;
  ScalaPQ pq;
  std::vector<const Read *> newRegions;
  int64_t mostRecentStart = 0;

  void checkSorted() {
    for (const Read *r : sorted) {
      if (r->start < mostRecentStart) fail(E_UNSORTED, "Regions must be sorted by start locus");
      mostRecentStart = r->start;
    }
  }
  void setCurrentLocus(int64_t locus) {  // :83-110
    if (!(locus >= currentLocus)) fail(E_ASSERT, "Pileup window can only move forward in locus");
    currentLocus = locus;
    while (!pq.empty() && pq.head()->end <= locus) pq.dequeue();
    newRegions.clear();
    while (next < sorted.size() && sorted[next]->start <= locus) {
      const Read *r = sorted[next++];
      if (r->overlapsLocus(locus)) newRegions.push_back(r);
    }
    for (const Read *r : newRegions) pq.enqueue(r);
  }
  bool nextLocusWithRegions(int64_t &out) const {  // :118-128
    for (size_t i = 1; i < pq.a.size(); ++i)
      if (pq.a[i]->overlapsLocus(currentLocus + 1)) {
        out = currentLocus + 1;
        return true;
      }
    if (next < sorted.size()) {
      out = std::max<int64_t>(0, sorted[next]->start);
      return true;
    }
    return false;
  }
  std::vector<const Read *> currentRegions() const { return std::vector<const Read *>(pq.a.begin() + 1, pq.a.end()); }
};

// LociSet.SingleContig.Iterator (LociSet.scala:287-351)
struct LociIter {
  std::vector<std::pair<int64_t, int64_t>> ranges;
  size_t ri = 0;
  int64_t idx = 0;
  bool hasNext() const { return ri < ranges.size(); }
  int64_t head() const { return ranges[ri].first + idx; }
  int64_t nextLocus() {
    int64_t r = head();
    ++idx;
    if (ranges[ri].first + idx >= ranges[ri].second) {
      ++ri;
      idx = 0;
    }
    return r;
  }
  void skipTo(int64_t locus) {
    while (ri < ranges.size() && ranges[ri].second <= locus) {
      ++ri;
      idx = 0;
    }
    if (ri < ranges.size() && locus >= ranges[ri].first && locus < ranges[ri].second) idx = locus - ranges[ri].first;
  }
};

// SlidingWindow.advanceMultipleWindows (SlidingWindow.scala:149-187), skipEmpty = true
bool advanceMultipleWindows(std::vector<Window *> &windows, LociIter &loci, int64_t &outLocus) {
  while (loci.hasNext()) {
    bool any = false;
    int64_t best = 0;
    for (Window *w : windows) {
      int64_t l;
      if (w->nextLocusWithRegions(l)) {
        if (!any || l < best) best = l;
        any = true;
      }
    }
    if (!any) return false;
    if (best <= loci.head()) {
      int64_t nl = loci.nextLocus();
      for (Window *w : windows) w->setCurrentLocus(nl);
      for (Window *w : windows)
        if (!w->pq.empty()) {
          outLocus = nl;
          return true;
        }
    } else {
      loci.skipTo(best);
    }
  }
  return false;
}

// pileup/Pileup.scala:37-186 -----------------------------------------------------------------
struct Pileup {
  int64_t locus = 0;
  uint8_t referenceBase = 'N';
  std::vector<Elem> elements;
  int depth() const { return (int)elements.size(); }
};

// Pileup.referenceBaseAtLocus (Pileup.scala:157-165): first read, in heap order, whose
// MD-derived base is standard.  `ambiguous` reports whether the reads disagree (i.e.
// whether heap order, not data, decides).
uint8_t referenceBaseAtLocus(const std::vector<const Read *> &reads, int64_t locus, bool *ambiguous) {
  uint8_t found = 'N';
  bool have = false;
  unsigned mask = 0;
  for (const Read *r : reads) {
    uint8_t b = r->referenceBaseAtLocus(locus);
    if (isStandardBase(b)) {
      if (!have) {
        found = b;
        have = true;
        if (!ambiguous) break;
      }
      mask |= 1u << (b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : 3);
    }
  }
  if (ambiguous) *ambiguous = __builtin_popcount(mask) > 1;
  return found;
}

// DistributedUtil.initOrMovePileup (DistributedUtil.scala:260-274) + Pileup.atGreaterLocus (Pileup.scala:103-132)
// ref_base >= 0: the reference genome's base (DistributedUtil.scala:266-267)
void initOrMovePileup(Pileup &p, bool exists, const Window &w, bool *ambiguous, int ref_base = -1) {
  int64_t locus = w.currentLocus;
  std::vector<const Read *> regions = w.currentRegions();
  uint8_t ref;
  if (ref_base >= 0) {
    ref = (uint8_t)ref_base;
    if (ambiguous) *ambiguous = false;
  } else {
    ref = referenceBaseAtLocus(regions, locus, ambiguous);
  }
  if (!exists) {
    p.locus = locus;
    p.referenceBase = ref;
    p.elements.clear();
    for (const Read *r : regions)
      if (r->overlapsLocus(locus)) p.elements.push_back(Elem::create(r, locus, ref));
    return;
  }
  if (!(p.elements.empty() || locus > p.locus)) fail(E_ASSERT, "New locus not greater than current locus");
  std::vector<Elem> out;
  out.reserve(p.elements.size() + w.newRegions.size());
  for (const Elem &e : p.elements)
    if (e.read->overlapsLocus(locus)) out.push_back(e.advanceToLocus(locus, ref));
  for (const Read *r : w.newRegions) out.push_back(Elem::create(r, locus, ref));
  p.elements.swap(out);
  p.locus = locus;
  p.referenceBase = ref;
}

// ------------------------------------------------------------------------------------------------
// Input marshalling
struct ReadSet {
  std::vector<Read> reads;
};

std::vector<CigarEl> decodeCigar(const uint32_t *c, int n) {
  std::vector<CigarEl> v((size_t)n);
  for (int i = 0; i < n; ++i) v[(size_t)i] = CigarEl{(int)(c[i] & 0xF), (int)(c[i] >> 4)};
  return v;
}

void buildReads(const or_reads *in, ReadSet &rs) {
  rs.reads.resize((size_t)in->n_reads);
  for (int64_t i = 0; i < in->n_reads; ++i) {
    Read &r = rs.reads[(size_t)i];
    r.index = i;
    r.contig = in->contig[i];
    r.start = in->start[i];
    r.mapq = in->mapq[i];
    r.positive = !(in->flags[i] & 1);
    r.sample = in->sample[i];
    r.sampleName = (r.sample >= 0 && r.sample < in->n_sample_names && in->sample_names && in->sample_names[r.sample])
                       ? std::string(in->sample_names[r.sample])
                       : std::string("default");
    r.seq = in->seq + in->seq_off[i];
    r.qual = in->qual + in->seq_off[i];
    r.len = in->seq_len[i];
    r.cigar = decodeCigar(in->cigar + in->cigar_off[i], in->n_cigar[i]);
    int64_t span = 0;
    for (const CigarEl &c : r.cigar)
      if (consumesRef(c.op) || c.op == OP_P) span += c.len;  // Cigar.getPaddedReferenceLength
    r.end = r.start + span;                                  // MappedRead.scala:87
    if (in->md_len[i] >= 0) {
      r.hasMd = true;
      r.md = parseMdTag(in->md + in->md_off[i], in->md_len[i], r.start, r.cigar);
    }
  }
}

struct TaskContig {
  int64_t task;
  int32_t contig;
  std::vector<std::pair<int64_t, int64_t>> ranges;
};

// Tasks x contigs in the order the reference's RDD emits them: task ascending, then
// contigs lexicographically (LociMap.scala:39-42), loci ascending.
std::vector<TaskContig> taskContigs(const or_loci *loci) {
  std::map<int64_t, std::map<std::string, TaskContig>> m;
  for (int64_t i = 0; i < loci->n_ranges; ++i) {
    if (loci->range_end[i] <= loci->range_start[i]) continue;
    int32_t c = loci->range_contig[i];
    auto &tc = m[loci->range_task[i]][loci->contig_names[c]];
    tc.task = loci->range_task[i];
    tc.contig = c;
    tc.ranges.push_back({loci->range_start[i], loci->range_end[i]});
  }
  std::vector<TaskContig> out;
  for (auto &t : m)
    for (auto &c : t.second) {
      auto &r = c.second.ranges;
      std::sort(r.begin(), r.end());
      // coalesce (LociMap.Builder.result)
      std::vector<std::pair<int64_t, int64_t>> merged;
      for (auto &x : r) {
        if (!merged.empty() && x.first <= merged.back().second) merged.back().second = std::max(merged.back().second, x.second);
        else merged.push_back(x);
      }
      c.second.ranges = merged;
      out.push_back(c.second);
    }
  return out;
}

// reads of `contig` assigned to a task: those overlapping any of the task's ranges
// (DistributedUtil.scala:585-597: getAll(start, end) with halfWindowSize = 0), in
// (start, input order) order (TaskPosition sort, stable).
std::vector<const Read *> taskReads(const ReadSet &rs, const std::vector<size_t> &byContigStart,
                                    const TaskContig &tc) {
  std::vector<const Read *> out;
  for (size_t idx : byContigStart) {
    const Read &r = rs.reads[idx];
    if (r.contig != tc.contig) continue;
    if (r.end <= r.start) continue;
    bool hit = false;
    auto it = std::upper_bound(tc.ranges.begin(), tc.ranges.end(), std::make_pair(r.start, INT64_MAX));
    if (it != tc.ranges.begin()) {
      auto p = std::prev(it);
      if (p->second > r.start) hit = true;
    }
    if (!hit && it != tc.ranges.end() && it->first < r.end) hit = true;
    if (hit) out.push_back(&r);
  }
  return out;
}

struct ContigIndex {  // per contig: read indices sorted by (start, input order)
  std::map<int32_t, std::vector<size_t>> by;
  explicit ContigIndex(const ReadSet &rs) {
    for (size_t i = 0; i < rs.reads.size(); ++i) by[rs.reads[i].contig].push_back(i);
    for (auto &kv : by)
      std::stable_sort(kv.second.begin(), kv.second.end(),
                       [&](size_t a, size_t b) { return rs.reads[a].start < rs.reads[b].start; });
  }
  const std::vector<size_t> &get(int32_t c) const {
    static const std::vector<size_t> empty;
    auto it = by.find(c);
    return it == by.end() ? empty : it->second;
  }
};

const char *gtName(int g) {
  switch (g) {
    case 0: return "Ref";
    case 1: return "Alt";
    case 2: return "OtherAlt";
    default: return "NoCall";
  }
}
enum { GT_REF = 0, GT_ALT = 1, GT_OTHERALT = 2, GT_NOCALL = 3 };

void appendf(std::string &s, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void appendf(std::string &s, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (n < (int)sizeof buf) {
    s.append(buf, (size_t)n);
  } else {
    std::string big((size_t)n + 1, '\0');
    va_start(ap, fmt);
    vsnprintf(&big[0], big.size(), fmt, ap);
    va_end(ap);
    s.append(big.data(), (size_t)n);
  }
}

// Pileup.bySample (Pileup.scala:57-61): elements.groupBy(sample name) then .map(...), so the
// samples come in the Scala Map's iteration order over their names (String.hashCode; the
// first occurrence in element order is the insertion order).  (sample slot, elements) pairs.
std::vector<std::pair<int, std::vector<const Elem *>>> bySampleOrdered(const Pileup &p) {
  std::vector<std::string> names;
  std::vector<std::pair<int, std::vector<const Elem *>>> groups;
  for (const Elem &e : p.elements) {
    size_t k = 0;
    while (k < names.size() && names[k] != e.read->sampleName) ++k;
    if (k == names.size()) {
      names.push_back(e.read->sampleName);
      groups.push_back({e.read->sample, {}});
    }
    groups[k].second.push_back(&e);
  }
  std::vector<uint32_t> hashes;
  for (const std::string &n : names) hashes.push_back(scala_order::javaStringHash(n));
  std::vector<std::pair<int, std::vector<const Elem *>>> out;
  for (int k : scala_order::groupByOrder(hashes)) out.push_back(groups[(size_t)k]);
  return out;
}

// GermlineThreshold.Caller.callVariantsAtLocus (GermlineThresholdCaller.scala:90-179)
void germlineCallAtLocus(const Pileup &p, const char *contig, int threshold, bool emitRef, bool emitNoCall,
                         bool ambiguousRef, std::string &out) {
  if (p.elements.empty()) return;
  // bySample (Pileup.scala:57-61): groupBy over the sample names, iterated in the Scala Map's order
  for (const auto &grp : bySampleOrdered(p)) {
    const int sampleSlot = grp.first;
    const auto &elems = grp.second;
    int total = (int)elems.size();
    // counts = elements.map(_.allele).groupBy(x => x).mapValues(_.length) (:103): the distinct
    // alleles in first-occurrence order, then the groupBy map's iteration order
    std::vector<Allele> distinct;
    std::vector<int> cnt;
    for (const Elem *e : elems) {
      const Allele &a = e->evaluate().allele;
      size_t k = 0;
      while (k < distinct.size() && !(distinct[k] == a)) ++k;
      if (k == distinct.size()) {
        distinct.push_back(a);
        cnt.push_back(0);
      }
      ++cnt[k];
    }
    std::vector<uint32_t> hashes;
    for (const Allele &a : distinct) hashes.push_back(scala_order::alleleHash(a));
    std::vector<std::pair<Allele, int>> sorted;
    for (int k : scala_order::groupByOrder(hashes))
      if ((int64_t)cnt[(size_t)k] * 100 / total > threshold) sorted.push_back({distinct[(size_t)k], cnt[(size_t)k]});
    // sortBy(-count) (:104): a stable sort, count ties keep the map's order
    std::stable_sort(sorted.begin(), sorted.end(),
                     [](const std::pair<Allele, int> &a, const std::pair<Allele, int> &b) { return a.second > b.second; });
    int flags = ambiguousRef ? 1 : 0;
    if (sorted.size() >= 2 && (sorted[0].second == sorted[1].second ||
                               (sorted.size() >= 3 && sorted[1].second == sorted[2].second)))
      flags |= 2;
    auto emit = [&](const std::string &ref, const std::string &alt, int g0, int g1) {
      appendf(out, "%s\t%lld\t%d\t%s,%s\t%s\t%s\t%d\n", contig, (long long)p.locus, sampleSlot, gtName(g0), gtName(g1),
              ref.c_str(), alt.c_str(), flags);
    };
    std::string refStr(1, (char)p.referenceBase);
    if (sorted.empty()) {
      if (emitNoCall) emit(refStr, "<ALT>", GT_NOCALL, GT_NOCALL);
    } else if (sorted.size() == 1 && !sorted[0].first.isVariant()) {
      if (emitRef) emit(refStr, "<ALT>", GT_REF, GT_REF);
    } else if (sorted.size() == 1) {
      emit(sorted[0].first.ref, sorted[0].first.alt, GT_ALT, GT_ALT);
    } else {
      const Allele &a1 = sorted[0].first, &a2 = sorted[1].first;
      if ((!a1.isVariant() || !a2.isVariant()) && (a1.alt.empty() ^ a2.alt.empty())) {
        // heterozygous deletion: no call
      } else if (a1.isVariant() ^ a2.isVariant()) {
        const Allele &v = a1.isVariant() ? a1 : a2;
        emit(v.ref, v.alt, GT_REF, GT_ALT);
      } else if (a1.isVariant() && a2.isVariant()) {
        emit(a1.ref, a1.alt, GT_ALT, GT_OTHERALT);
        emit(a2.ref, a2.alt, GT_ALT, GT_OTHERALT);
      } else {
        if (a1.ref == "N" || a2.ref == "N") {
          const std::string &proper = a1.ref == "N" ? a2.ref : a1.ref;
          emit(proper, "<ALT>", GT_REF, GT_REF);
        } else {
          fail(E_MULTI_REF, std::string("Multiple reference bases found at ") + contig + ":" + std::to_string(p.locus));
        }
      }
    }
  }
}

// Drives pileupFlatMap / pileupFlatMapTwoRDDs (DistributedUtil.scala:288-335, 388-418, 473-486)
// ReferenceBroadcast.getReferenceBase (ReferenceBroadcast.scala:26-37): ContigNotFound for a
// contig the reference lacks, an index failure past its end
int referenceBase(const or_reference *ref, const or_loci *loci, int32_t contig, int64_t locus) {
  if (contig < 0 || contig >= ref->n_contigs || !ref->bases[contig])
    fail(E_ARG, std::string("Contig ") + loci->contig_names[contig] + " does not exist in the current reference");
  if (locus < 0 || locus >= ref->lengths[contig])
    fail(E_ARG, std::string("locus ") + std::to_string(locus) + " is past the end of reference contig " +
                    loci->contig_names[contig]);
  return ref->bases[contig][locus];
}

template <class F>
void forEachPileup(const std::vector<ReadSet *> &sets, const or_loci *loci, F &&fn,
                   const or_reference *reference = nullptr) {
  std::vector<ContigIndex> idx;
  for (ReadSet *rs : sets) idx.emplace_back(*rs);
  for (const TaskContig &tc : taskContigs(loci)) {
    std::vector<Window> windows(sets.size());
    for (size_t s = 0; s < sets.size(); ++s) {
      windows[s].sorted = taskReads(*sets[s], idx[s].get(tc.contig), tc);
      windows[s].checkSorted();
    }
    std::vector<Window *> wp;
    for (auto &w : windows) wp.push_back(&w);
    LociIter it;
    it.ranges = tc.ranges;
    std::vector<Pileup> pileups(sets.size());
    bool have = false;
    int64_t locus;
    while (advanceMultipleWindows(wp, it, locus)) {
      std::vector<bool> amb(sets.size(), false);
      const int rb = reference ? referenceBase(reference, loci, tc.contig, locus) : -1;
      for (size_t s = 0; s < sets.size(); ++s) {
        bool a = false;
        initOrMovePileup(pileups[s], have, windows[s], &a, rb);
        amb[s] = a;
      }
      have = true;
      fn(tc, pileups, amb);
    }
  }
}

int guard(std::string &out, char **o, int64_t *olen, const std::function<void()> &body) {
  try {
    body();
  } catch (const OracleError &e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception &e) {
    g_err = e.what();
    return E_ASSERT;
  }
  char *p = (char *)malloc(out.size() + 1);
  memcpy(p, out.data(), out.size());
  p[out.size()] = 0;
  *o = p;
  *olen = (int64_t)out.size();
  return 0;
}

// ---- somatic: filters/PileupFilter.scala:29-89, likelihood/Likelihood.scala:48-201,
//      variants/AlleleEvidence.scala:41-102, commands/SomaticStandardCaller.scala:162-245
struct Genotype {
  Allele a1, a2;
  bool hasVariantAllele() const { return a1.isVariant() || a2.isVariant(); }
};

std::vector<const Elem *> pileupFilter(const Pileup &p, bool filterMultiAllelic, int minMapq) {
  std::vector<const Elem *> els;
  for (const Elem &e : p.elements) els.push_back(&e);
  if (filterMultiAllelic) {
    std::vector<Allele> d;
    for (const Elem *e : els) {
      const Allele &a = e->evaluate().allele;
      if (std::find(d.begin(), d.end(), a) == d.end()) d.push_back(a);
    }
    if (d.size() > 2) els.clear();
  }
  if (minMapq > 0) {
    std::vector<const Elem *> k;
    for (const Elem *e : els)
      if (e->read->mapq >= minMapq) k.push_back(e);
    els.swap(k);
  }
  return els;
}

std::vector<double> likelihoodsOfGenotypes(const std::vector<const Elem *> &elements,
                                           const std::vector<Genotype> &genotypes, bool includeAlignment,
                                           bool normalize, bool logSpace = false) {
  std::vector<Allele> alleles;
  for (const Genotype &g : genotypes) {
    for (const Allele *a : {&g.a1, &g.a2})
      if (std::find(alleles.begin(), alleles.end(), *a) == alleles.end()) alleles.push_back(*a);
  }
  std::sort(alleles.begin(), alleles.end());
  size_t depth = elements.size();
  std::vector<std::vector<double>> m(alleles.size(), std::vector<double>(depth));
  for (size_t ai = 0; ai < alleles.size(); ++ai)
    for (size_t ei = 0; ei < depth; ++ei) {
      const Elem *e = elements[ei];
      double pc = phredToSuccessProbability(e->evaluate().quality);
      if (includeAlignment) pc = pc * e->read->alignmentLikelihood();
      m[ai][ei] = (alleles[ai] == e->evaluate().allele) ? pc : 1 - pc;
    }
  auto indexOf = [&](const Allele &a) { return (size_t)(std::find(alleles.begin(), alleles.end(), a) - alleles.begin()); };
  std::vector<double> ll;
  for (const Genotype &g : genotypes) {
    const auto &r1 = m[indexOf(g.a1)];
    const auto &r2 = m[indexOf(g.a2)];
    double agg;
    if (depth == 0) agg = NAN;  // Colt aggregate of an empty vector
    else {
      agg = strictmath::log(r1[depth - 1] + r2[depth - 1]);
      for (size_t i = depth - 1; i-- > 0;) agg = agg + strictmath::log(r1[i] + r2[i]);
    }
    ll.push_back(agg + strictmath::log(1.0) - strictmath::log(2.0) * (double)depth);
  }
  if (normalize) {
    double tot = 0.0;
    for (double x : ll) tot += strictmath::exp(x);
    double lt = strictmath::log(tot);
    for (double &x : ll) x = x - lt;
  }
  if (!logSpace)
    for (double &x : ll) x = strictmath::exp(x);
  return ll;
}

std::vector<std::pair<Genotype, double>> likelihoodsOfAllPossibleGenotypes(const std::vector<const Elem *> &els,
                                                                           bool includeAlignment,
                                                                           bool normalize = true,
                                                                           bool logSpace = false) {
  std::vector<Allele> distinct;
  for (const Elem *e : els) {
    const Allele &a = e->evaluate().allele;
    if (std::find(distinct.begin(), distinct.end(), a) == distinct.end()) distinct.push_back(a);
  }
  std::sort(distinct.begin(), distinct.end());
  std::vector<Allele> alleles;
  for (const Allele &a : distinct) {
    bool ok = true;
    for (char c : a.alt) ok = ok && isStandardBase((uint8_t)c);
    if (ok) alleles.push_back(a);
  }
  std::vector<Genotype> gts;
  for (size_t i = 0; i < alleles.size(); ++i)
    for (size_t j = i; j < alleles.size(); ++j) gts.push_back(Genotype{alleles[i], alleles[j]});
  std::vector<double> l = likelihoodsOfGenotypes(els, gts, includeAlignment, normalize, logSpace);
  std::vector<std::pair<Genotype, double>> out;
  for (size_t i = 0; i < gts.size(); ++i) out.push_back({gts[i], l[i]});
  return out;
}

struct Evidence {
  double likelihood;
  int readDepth, alleleReadDepth, forwardDepth, alleleForwardDepth;
  double meanMQ, medianMQ, meanBQ, medianBQ, medianMismatches;
  int phred() const { return successProbabilityToPhred(likelihood - 1e-10); }
  float vaf() const { return (float)alleleReadDepth / (float)readDepth; }
};

double breezeMean(const std::vector<double> &v) {  // breeze.stats.mean (running mean)
  double mu = 0.0;
  for (size_t i = 0; i < v.size(); ++i) mu += (v[i] - mu) / (double)(i + 1);
  return mu;
}
double breezeMedian(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  size_t n = v.size();
  if (n % 2 == 1) return v[(n - 1) / 2];
  return (v[n / 2 - 1] + v[n / 2]) / 2.0;
}
int breezeMedianInt(std::vector<int> v) {  // Int vector: integer arithmetic (parity unpinned for even n)
  std::sort(v.begin(), v.end());
  size_t n = v.size();
  if (n % 2 == 1) return v[(n - 1) / 2];
  return (v[n / 2 - 1] + v[n / 2]) / 2;
}

Evidence alleleEvidence(double likelihood, const Allele &allele, const std::vector<const Elem *> &els) {
  Evidence ev{};
  ev.likelihood = likelihood;
  ev.readDepth = (int)els.size();
  std::vector<double> mq, bq;
  std::vector<int> mm;
  for (const Elem *e : els) {
    if (e->read->positive) ev.forwardDepth++;
    if (e->evaluate().allele == allele) {
      ev.alleleReadDepth++;
      if (e->read->positive) ev.alleleForwardDepth++;
      mq.push_back((double)e->read->mapq);
      bq.push_back((double)e->evaluate().quality);
      if (!e->read->hasMd) fail(E_NO_MD, "None.get (mdTagOpt) for countOfMismatches");
      mm.push_back(e->read->md.countOfMismatches());
    }
  }
  if (mq.empty()) {
    ev.meanMQ = ev.medianMQ = ev.meanBQ = ev.medianBQ = ev.medianMismatches = NAN;
  } else {
    ev.meanMQ = breezeMean(mq);
    ev.medianMQ = breezeMedian(mq);
    ev.meanBQ = breezeMean(bq);
    ev.medianBQ = breezeMedian(bq);
    ev.medianMismatches = (double)breezeMedianInt(mm);
  }
  return ev;
}

void appendEvidence(std::string &out, const Evidence &e) {
  appendf(out, "\t%.17g\t%d\t%d\t%d\t%d\t%.17g\t%.17g\t%.17g\t%.17g\t%.17g", e.likelihood, e.readDepth,
          e.alleleReadDepth, e.forwardDepth, e.alleleForwardDepth, e.meanMQ, e.medianMQ, e.meanBQ, e.medianBQ,
          e.medianMismatches);
}


// Pileup.apply(reads, referenceName, locus) (Pileup.scala:181-186)
Pileup pileupApply(const ReadSet &rs, int32_t contig, int64_t locus) {
  std::vector<const Read *> overlapping;
  for (const Read &r : rs.reads)
    if (r.contig == contig && r.overlapsLocus(locus)) overlapping.push_back(&r);
  Pileup p;
  p.locus = locus;
  p.referenceBase = referenceBaseAtLocus(overlapping, locus, nullptr);
  for (const Read *r : overlapping) p.elements.push_back(Elem::create(r, locus, p.referenceBase));
  return p;
}
const char *kindName(Kind k) {
  static const char *n[] = {"Match", "Mismatch", "Insertion", "Deletion", "MidDeletion", "Clipped"};
  return n[k];
}
Allele parseAllele(const std::string &s) {
  size_t c = s.find(',');
  if (c == std::string::npos) fail(E_ARG, "bad allele spec " + s);
  return Allele{s.substr(0, c), s.substr(c + 1)};
}
std::vector<std::string> split(const std::string &s, char d) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    size_t e = s.find(d, b);
    out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) break;
    b = e + 1;
  }
  return out;
}

// SomaticStandard.Caller.findPotentialVariantAtLocus (SomaticStandardCaller.scala:162-245) and the
// filters: filterMode 1 = driver chain (:124-151 + SomaticGenotypeFilter.apply(RDD) :285-307),
// 2 = Seq form used by the reference's test suite (SomaticGenotypeFilter.scala:313-337).
void somaticAtLocus(const Pileup &tp, const Pileup &np, const char *contigName, const or_somatic_params *prm,
                    int filterMode, int flags, std::string &out) {
      auto fn = pileupFilter(np, prm->filter_multi_allelic != 0, prm->min_mapq);
      auto ft = pileupFilter(tp, prm->filter_multi_allelic != 0, prm->min_mapq);
      int tRefDepth = 0;
      for (const Elem *e : ft)
        if (e->evaluate().kind == K_MATCH) ++tRefDepth;
      if (ft.empty() || fn.empty() || (int64_t)ft.size() > prm->max_read_depth ||
          (int64_t)fn.size() > prm->max_read_depth || tRefDepth == (int)ft.size())
        return;
      auto tg = likelihoodsOfAllPossibleGenotypes(ft, true);
      if (tg.empty()) return;
      size_t best = 0;  // maxBy: first maximum
      for (size_t i = 1; i < tg.size(); ++i)
        if (tg[i].second > tg[best].second) best = i;
      const Genotype &mlg = tg[best].first;
      double mll = tg[best].second;
      if (!mlg.hasVariantAllele()) return;
      auto ng = likelihoodsOfAllPossibleGenotypes(fn, false);
      // normalLikelihoods.toMap.filter(_._1.hasVariantAllele).map(_._2).sum (:206-217): the
      // genotypes in the immutable Map's order (insertion order up to four, else HashTrieMap)
      std::vector<size_t> gorder(ng.size());
      for (size_t i = 0; i < ng.size(); ++i) gorder[i] = i;
      if (ng.size() > 4)
        std::stable_sort(gorder.begin(), gorder.end(), [&](size_t a, size_t b) {
          return scala_order::trieKey(scala_order::genotypeHash(ng[a].first.a1, ng[a].first.a2)) <
                 scala_order::trieKey(scala_order::genotypeHash(ng[b].first.a1, ng[b].first.a2));
        });
      double nvs = 0.0;
      for (size_t i : gorder)
        if (ng[i].first.hasVariantAllele()) nvs += ng[i].second;
      double odds = mll / nvs;
      if (!(odds * 100 >= prm->odds)) return;
      // test-infrastructure flag (same rule as the device, GQ_FLAG_KNIFE_EDGE = 4): a decision
      // within FP rounding of its threshold depends on summation order in the reference itself
      auto nearEdge = [](double a, double b) { return std::fabs(a - b) <= 1e-9 * std::max(1.0, std::fabs(b)); };
      if (nearEdge(odds * 100, prm->odds)) flags |= 4;
      const Allele *allele = nullptr;
      for (const Allele *a : {&mlg.a1, &mlg.a2})
        if (a->isVariant() && !a->alt.empty()) {
          allele = a;
          break;
        }
      if (!allele) return;
      Evidence tev = alleleEvidence(mll, *allele, ft);
      Evidence nev = alleleEvidence(1 - nvs, Allele{allele->ref, allele->ref}, fn);
      double logOdds = strictmath::log(odds);
      int gq = successProbabilityToPhred(tev.likelihood * nev.likelihood - 1e-10);
      {
        double x = -10.0 * strictmath::log10(1.0 - (tev.likelihood * nev.likelihood - 1e-10));
        if (std::isfinite(x) && std::fabs((x - std::floor(x)) - 0.5) <= 1e-6) flags |= 4;
      }
      if (filterMode == 1) {
        // SomaticStandardCaller.scala:124-137 then SomaticGenotypeFilter.apply (:285-307)
        auto depthOk = [&]() {
          return tev.readDepth >= prm->min_tumor_read_depth && tev.readDepth < prm->max_tumor_read_depth &&
                 nev.readDepth >= prm->min_normal_read_depth && nev.readDepth < INT32_MAX;
        };
        if (!depthOk()) return;
        if (!(tev.alleleReadDepth >= prm->min_tumor_alternate_read_depth)) return;
        if (!depthOk()) return;
        if (prm->min_tumor_alternate_read_depth > 0 && !(tev.alleleReadDepth >= prm->min_tumor_alternate_read_depth))
          return;
        if (!(logOdds > prm->min_lod)) return;
        if (nearEdge(logOdds, prm->min_lod)) flags |= 4;
        if (!(gq >= prm->min_likelihood)) return;
        if (!((double)tev.vaf() * 100.0 > prm->min_vaf)) return;
        if (!(tev.meanMQ >= prm->min_average_mapping_quality && nev.meanMQ >= prm->min_average_mapping_quality))
          return;
        if (nearEdge(tev.meanMQ, prm->min_average_mapping_quality) || nearEdge(nev.meanMQ, prm->min_average_mapping_quality) ||
            nearEdge(tev.meanMQ, prm->min_average_base_quality) || nearEdge(nev.meanMQ, prm->min_average_base_quality))
          flags |= 4;
        if (!(tev.meanMQ >= prm->min_average_base_quality && nev.meanMQ >= prm->min_average_base_quality)) return;
        if (!(tev.medianMismatches <= prm->max_median_mismatches)) return;
      }
      if (filterMode == 2) {
        if (!(tev.readDepth >= prm->min_tumor_read_depth && tev.readDepth < prm->max_tumor_read_depth &&
              nev.readDepth >= prm->min_normal_read_depth && nev.readDepth < INT32_MAX))
          return;
        if (!((double)tev.vaf() * 100.0 > prm->min_vaf)) return;
        if (!(gq >= prm->min_likelihood)) return;
        if (prm->min_tumor_alternate_read_depth > 0 && !(tev.alleleReadDepth >= prm->min_tumor_alternate_read_depth))
          return;
      }
      int sample = tp.elements.empty() ? 0 : tp.elements[0].read->sample;
      appendf(out, "%s\t%lld\t%d\t%s\t%s\t%.17g\t%d", contigName, (long long)tp.locus, sample,
              allele->ref.c_str(), allele->alt.c_str(), logOdds, gq);
      appendEvidence(out, tev);
      appendEvidence(out, nev);
      appendf(out, "\t%d\n", flags);
}
// GermlineStandard.Caller.callVariantsAtLocus (commands/GermlineStandardCaller.scala:90-124) +
// GenotypeFilter (filters/GenotypeFilter.scala:140-154) when apply_filters.  Per sample of the
// pileup (bySample: a Scala Map; here by sample index, unpinned for > 1 sample): the elements
// passing QualityAlignedReadsFilter, the ML genotype over likelihoodsOfAllPossibleGenotypes
// (log space, normalized; maxBy keeps the first maximum), probability = exp of it, and for each
// non-reference allele of the genotype (both, for a hom-alt) the allele's evidence over the
// sample's unfiltered elements.  Lines as somatic-standard's (normal evidence zero, log-odds 0,
// gq = the evidence's phredScaledLikelihood).
void germlineStandardAtLocus(const Pileup &p, const char *contigName, const or_germline_std_params *prm,
                             bool ambiguousRef, std::string &out) {
  if (p.elements.empty()) return;
  std::map<int, std::vector<const Elem *>> bySample;
  for (const Elem &e : p.elements) bySample[e.read->sample].push_back(&e);
  for (auto &kv : bySample) {
    const std::vector<const Elem *> &all = kv.second;
    std::vector<const Elem *> filt;
    for (const Elem *e : all)
      if (e->read->mapq >= prm->min_mapq) filt.push_back(e);  // QualityAlignedReadsFilter
    if (filt.empty()) continue;
    auto gl = likelihoodsOfAllPossibleGenotypes(filt, false, true, true);
    if (gl.empty()) fail(E_ASSERT, "empty.maxBy");
    size_t best = 0;
    for (size_t i = 1; i < gl.size(); ++i)
      if (gl[i].second > gl[best].second) best = i;
    const double probability = strictmath::exp(gl[best].second);
    const Genotype &g = gl[best].first;
    for (const Allele *a : {&g.a1, &g.a2}) {
      if (!a->isVariant()) continue;
      Evidence ev = alleleEvidence(probability, *a, all);
      const int gq = successProbabilityToPhred(ev.likelihood - 1e-10);
      if (prm->apply_filters) {
        if (!(ev.readDepth >= prm->min_read_depth && ev.readDepth < prm->max_read_depth)) continue;
        if (prm->min_alternate_read_depth > 0 && !(ev.alleleReadDepth >= prm->min_alternate_read_depth)) continue;
        if (prm->min_likelihood > 0 && !(gq >= prm->min_likelihood)) continue;
      }
      appendf(out, "%s\t%lld\t%d\t%s\t%s\t%.17g\t%d", contigName, (long long)p.locus, kv.first, a->ref.c_str(),
              a->alt.c_str(), 0.0, gq);
      appendEvidence(out, ev);
      appendEvidence(out, Evidence{});
      appendf(out, "\t%d\n", ambiguousRef ? 1 : 0);  // bit0: heap-order reference base
    }
  }
}
}  // namespace

extern "C" {

int or_germline_standard(const or_reads *reads, const or_loci *loci, const or_germline_std_params *prm, char **o,
                         int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    std::vector<ReadSet *> sets{&rs};
    forEachPileup(sets, loci, [&](const TaskContig &tc, std::vector<Pileup> &ps, std::vector<bool> &amb) {
      germlineStandardAtLocus(ps[0], loci->contig_names[tc.contig], prm, amb[0], out);
    });
  });
}

const char *or_last_error(void) { return g_err.c_str(); }
void or_scala_group_order(const uint32_t *hashes, int32_t n, int32_t *out) {
  std::vector<uint32_t> h(hashes, hashes + n);
  const std::vector<int> o = scala_order::groupByOrder(h);
  for (int32_t i = 0; i < n; ++i) out[i] = o[(size_t)i];
}
uint32_t or_scala_allele_hash(const char *ref, const char *alt) {
  return scala_order::alleleHash(Allele{ref, alt});
}
uint32_t or_scala_genotype_hash(const char *r1, const char *a1, const char *r2, const char *a2) {
  return scala_order::genotypeHash(Allele{r1, a1}, Allele{r2, a2});
}

void or_free(char *p) { free(p); }

int or_pileup_stats(const or_reads *reads, const or_loci *loci, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    std::vector<ReadSet *> sets{&rs};
    forEachPileup(sets, loci, [&](const TaskContig &tc, std::vector<Pileup> &ps, std::vector<bool> &amb) {
      const Pileup &p = ps[0];
      int pos = 0, refDepth = 0;
      int base[6] = {0, 0, 0, 0, 0, 0};
      int ins = 0, del = 0, mid = 0, clip = 0;
      for (const Elem &e : p.elements) {
        if (e.read->positive) ++pos;
        const Evaluated &ev = e.evaluate();
        switch (ev.kind) {
          case K_MATCH:
          case K_MISMATCH: {
            uint8_t b = (uint8_t)ev.allele.alt[0];
            int k = b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : b == 'T' ? 3 : b == 'N' ? 4 : 5;
            base[k]++;
            if (ev.kind == K_MATCH) ++refDepth;
            break;
          }
          case K_INSERTION: ++ins; break;
          case K_DELETION: ++del; break;
          case K_MIDDELETION: ++mid; break;
          case K_CLIPPED: ++clip; break;
        }
      }
      appendf(out, "%s\t%lld\t%c\t%d\t%d\t%d %d %d %d %d %d\t%d %d %d %d\t%d\t%d\n", loci->contig_names[tc.contig],
              (long long)p.locus, (char)p.referenceBase, p.depth(), pos, base[0], base[1], base[2], base[3], base[4],
              base[5], ins, del, mid, clip, refDepth, amb[0] ? 1 : 0);
    });
  });
}

int or_heap_orders(const or_reads *const *reads, int32_t n_sets, const or_loci *loci, int64_t every, char **o,
                   int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    std::vector<ReadSet> rs((size_t)n_sets);
    std::vector<ContigIndex> idx;
    for (int32_t s = 0; s < n_sets; ++s) {
      buildReads(reads[s], rs[(size_t)s]);
      idx.emplace_back(rs[(size_t)s]);
    }
    for (const TaskContig &tc : taskContigs(loci)) {
      std::vector<Window> windows((size_t)n_sets);
      std::vector<Window *> wp;
      for (int32_t s = 0; s < n_sets; ++s) {
        windows[(size_t)s].sorted = taskReads(rs[(size_t)s], idx[(size_t)s].get(tc.contig), tc);
        windows[(size_t)s].checkSorted();
        wp.push_back(&windows[(size_t)s]);
      }
      LociIter it;
      it.ranges = tc.ranges;
      int64_t locus;
      while (advanceMultipleWindows(wp, it, locus)) {
        if (every > 1 && locus % every != 0) continue;
        for (int32_t s = 0; s < n_sets; ++s) {
          appendf(out, "%d\t%lld\t%d\t", tc.contig, (long long)locus, s);
          const auto regions = windows[(size_t)s].currentRegions();
          for (size_t k = 0; k < regions.size(); ++k) appendf(out, k ? ",%lld" : "%lld", (long long)regions[k]->index);
          out.push_back('\n');
        }
      }
    }
  });
}

int or_germline_threshold(const or_reads *reads, const or_loci *loci, int32_t threshold, int32_t emit_ref,
                          int32_t emit_no_call, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    std::vector<ReadSet *> sets{&rs};
    forEachPileup(sets, loci, [&](const TaskContig &tc, std::vector<Pileup> &ps, std::vector<bool> &amb) {
      germlineCallAtLocus(ps[0], loci->contig_names[tc.contig], threshold, emit_ref != 0, emit_no_call != 0, amb[0],
                          out);
    });
  });
}

int or_somatic_standard_ref(const or_reads *tumor, const or_reads *normal, const or_loci *loci,
                            const or_reference *ref, const or_somatic_params *prm, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet trs, nrs;
    buildReads(tumor, trs);
    buildReads(normal, nrs);
    std::vector<ReadSet *> sets{&trs, &nrs};
    forEachPileup(
        sets, loci,
        [&](const TaskContig &tc, std::vector<Pileup> &ps, std::vector<bool> &amb) {
          somaticAtLocus(ps[0], ps[1], loci->contig_names[tc.contig], prm, prm->apply_filters,
                         (amb[0] ? 1 : 0) | (amb[1] ? 2 : 0), out);
        },
        ref);
  });
}

int or_somatic_standard(const or_reads *tumor, const or_reads *normal, const or_loci *loci,
                        const or_somatic_params *prm, char **o, int64_t *olen) {
  return or_somatic_standard_ref(tumor, normal, loci, nullptr, prm, o, olen);
}

// VariantSupport.pileupToAlleleCounts (commands/VariantSupport.scala:110-118) over
// pileupFlatMap(reads, partitions, skipEmpty = true) (:93-100): per pileup, the elements
// grouped by allele.  Rows: sample of the head element (Pileup.sampleName, Pileup.scala:51),
// contig, locus, ref, alt, count, flags (bit0: heap-order reference base); within a locus by
// (ref, alt) — the reference iterates a Scala HashMap there (order unpinned).
int or_variant_support(const or_reads *reads, const or_loci *loci, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    std::vector<ReadSet *> sets{&rs};
    forEachPileup(sets, loci, [&](const TaskContig &tc, std::vector<Pileup> &ps, std::vector<bool> &amb) {
      const Pileup &p = ps[0];
      if (p.elements.empty()) return;
      std::map<std::pair<std::string, std::string>, int> counts;
      for (const Elem &e : p.elements) {
        const Evaluated &ev = e.evaluate();
        ++counts[{ev.allele.ref, ev.allele.alt}];
      }
      for (const auto &kv : counts)
        appendf(out, "%d\t%s\t%lld\t%s\t%s\t%d\t%d\n", p.elements.front().read->sample,
                loci->contig_names[tc.contig], (long long)p.locus, kv.first.first.c_str(), kv.first.second.c_str(),
                kv.second, amb[0] ? 1 : 0);
    });
  });
}

// VAFHistogram (commands/VAFHistogram.scala:31-37, 188-229): per non-empty pileup with a
// non-Match element, VAF = (depth - referenceDepth).toFloat / depth (referenceDepth = Match
// elements, Pileup.scala:86-91), kept for depth >= minReadDepth and VAF >= minVAF / 100.0,
// binned as pct - pct % (100 / bins), pct = (VAF * 100).toInt.  Lines: bin \t loci, then
// "variant \t N".
int or_vaf_histogram(const or_reads *reads, const or_loci *loci, int32_t bins, int32_t min_read_depth,
                     int32_t min_vaf, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    if (!(bins <= 100 && bins >= 1)) fail(E_ASSERT, "assumption failed: Bins should be between 1 and 100");
    ReadSet rs;
    buildReads(reads, rs);
    std::vector<ReadSet *> sets{&rs};
    std::map<int, int64_t> hist;
    int64_t variant = 0;
    const int bin_size = 100 / bins;
    forEachPileup(sets, loci, [&](const TaskContig &, std::vector<Pileup> &ps, std::vector<bool> &) {
      const Pileup &p = ps[0];
      const int depth = p.depth();
      int ref = 0;
      for (const Elem &e : p.elements)
        if (e.evaluate().kind == K_MATCH) ++ref;
      if (ref == depth) return;
      const float vaf = (float)(depth - ref) / (float)depth;
      if (!(depth >= min_read_depth) || !((double)vaf >= (double)min_vaf / 100.0)) return;
      const int pct = (int)(vaf * 100.0f);
      ++hist[pct - pct % bin_size];
      ++variant;
    });
    for (const auto &kv : hist) appendf(out, "%d\t%lld\n", kv.first, (long long)kv.second);
    appendf(out, "variant\t%lld\n", (long long)variant);
  });
}

int or_elements_at(const or_reads *reads, int32_t contig, int64_t locus, int32_t own_ref, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    std::vector<Elem> els;
    uint8_t ref = 'N';
    if (own_ref) {  // PileupSuite.pileupElementFromRead: PileupElement(read, locus, read.getReferenceBaseAtLocus(locus))
      for (const Read &r : rs.reads) {
        uint8_t b = r.referenceBaseAtLocus(locus);
        els.push_back(Elem::create(&r, locus, b));
        ref = b;
      }
    } else {
      Pileup p = pileupApply(rs, contig, locus);
      els = p.elements;
      ref = p.referenceBase;
    }
    appendf(out, "ref\t%c\n", (char)ref);
    for (const Elem &e : els) {
      const Evaluated &ev = e.evaluate();
      appendf(out, "%lld\t%s\t%s\t%s\t%d\t%d\t%d\t%d\n", (long long)e.read->index, kindName(ev.kind),
              ev.allele.ref.c_str(), ev.allele.alt.c_str(), ev.quality, e.readPosition, e.cigarElementIndex,
              e.indexWithinCigarElement);
    }
  });
}

int or_likelihoods_at(const or_reads *reads, int32_t contig, int64_t locus, const char *spec, int32_t include_alignment,
                      int32_t log_space, int32_t normalize, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    Pileup p = pileupApply(rs, contig, locus);
    std::vector<const Elem *> els;
    for (const Elem &e : p.elements) els.push_back(&e);
    std::vector<std::pair<Genotype, double>> res;
    std::string sp = spec ? spec : "";
    if (sp.empty()) {
      res = likelihoodsOfAllPossibleGenotypes(els, include_alignment != 0, normalize != 0, log_space != 0);
    } else {
      std::vector<Genotype> gts;
      for (const std::string &g : split(sp, '|')) {
        auto al = split(g, ';');
        if (al.size() != 2) fail(E_ARG, "Non-diploid genotype not supported");
        gts.push_back(Genotype{parseAllele(al[0]), parseAllele(al[1])});
      }
      auto l = likelihoodsOfGenotypes(els, gts, include_alignment != 0, normalize != 0, log_space != 0);
      for (size_t i = 0; i < gts.size(); ++i) res.push_back({gts[i], l[i]});
    }
    for (auto &r : res)
      appendf(out, "%s,%s;%s,%s\t%.17g\n", r.first.a1.ref.c_str(), r.first.a1.alt.c_str(), r.first.a2.ref.c_str(),
              r.first.a2.alt.c_str(), r.second);
  });
}

int or_allele_evidence_at(const or_reads *reads, int32_t contig, int64_t locus, double likelihood, const char *ref,
                          const char *alt, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    Pileup p = pileupApply(rs, contig, locus);
    std::vector<const Elem *> els;
    for (const Elem &e : p.elements) els.push_back(&e);
    Evidence ev = alleleEvidence(likelihood, Allele{ref, alt}, els);
    appendEvidence(out, ev);
    out += "\n";
  });
}

int or_germline_at(const or_reads *reads, int32_t contig, int64_t locus, int32_t threshold, int32_t emit_ref,
                   int32_t emit_no_call, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet rs;
    buildReads(reads, rs);
    Pileup p = pileupApply(rs, contig, locus);
    germlineCallAtLocus(p, "contig", threshold, emit_ref != 0, emit_no_call != 0, false, out);
  });
}

int or_somatic_at(const or_reads *tumor, const or_reads *normal, int32_t contig, int64_t locus,
                  const or_somatic_params *prm, char **o, int64_t *olen) {
  std::string out;
  return guard(out, o, olen, [&]() {
    ReadSet trs, nrs;
    buildReads(tumor, trs);
    buildReads(normal, nrs);
    Pileup tp = pileupApply(trs, contig, locus), np = pileupApply(nrs, contig, locus);
    somaticAtLocus(tp, np, "contig", prm, prm->apply_filters, 0, out);
  });
}

}  // extern "C"
