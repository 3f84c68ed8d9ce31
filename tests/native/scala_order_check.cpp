// Host build of guacamole_amd/csrc/gq_scala_order.h for tests/test_scala_order.py: reads
// "ref alt" lines ("-" = empty) and prints the allele hash, its 16-bucket index and trie key.
#include <cstdio>
#include <iostream>
#include <string>

#include "gq_scala_order.h"

int main() {
  std::string r, a;
  while (std::cin >> r >> a) {
    if (r == "-") r.clear();
    if (a == "-") a.clear();
    gq::scala::SeqHasher hr, ha;
    for (unsigned char c : r) hr.add_byte(c);
    for (unsigned char c : a) ha.add_byte(c);
    const uint32_t h = gq::scala::allele_hash(hr.result(), ha.result());
    std::printf("%u %u %llu\n", h, gq::scala::mutable_bucket(h, 4), (unsigned long long)gq::scala::trie_key(h));
  }
  return 0;
}
