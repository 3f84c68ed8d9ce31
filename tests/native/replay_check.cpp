// Host build of the product's heap replay (guacamole_amd/csrc/gq_replay.h) for
// tests/test_replay.py, which compares it with the oracle's SlidingWindow restatement.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../guacamole_amd/csrc/gq_replay.h"

extern "C" {
// sets: n_sets read sets of one contig (index order): n[s], start/end/pmax[s], lo[s] (absolute
// index of the first); window ranges; sorted query loci.  Output text: "locus\tset\tr,r,..\n".
int rp_replay(int n_sets, const int64_t *n, const int32_t *const *start, const int32_t *const *end,
              const int32_t *const *pmax, const int64_t *lo, int64_t n_ranges, const int64_t *rs,
              const int64_t *re, int64_t n_q, const int32_t *qpos, char **out, int64_t *out_len) {
  std::vector<gq::ReplaySet> sets((size_t)n_sets);
  for (int s = 0; s < n_sets; ++s) {
    sets[(size_t)s].lo = lo[s];
    sets[(size_t)s].start.assign(start[s], start[s] + n[s]);
    sets[(size_t)s].end.assign(end[s], end[s] + n[s]);
    sets[(size_t)s].pmax.assign(pmax[s], pmax[s] + n[s]);
  }
  std::vector<int64_t> vrs(rs, rs + n_ranges), vre(re, re + n_ranges);
  std::vector<gq::ReplayQuery> qs;
  for (int64_t i = 0; i < n_q; ++i) qs.push_back(gq::ReplayQuery{qpos[i], (int32_t)i});
  std::string o;
  gq::replay_heaps(vrs, vre, sets, qs, [&](int32_t id, int k, const int64_t *h, int64_t nh) {
    o += std::to_string(qpos[id]) + "\t" + std::to_string(k) + "\t";
    for (int64_t i = 0; i < nh; ++i) {
      if (i) o += ",";
      o += std::to_string(h[i]);
    }
    o += "\n";
  });
  *out = (char *)malloc(o.size() + 1);
  memcpy(*out, o.data(), o.size());
  (*out)[o.size()] = 0;
  *out_len = (int64_t)o.size();
  return 0;
}
void rp_free(char *p) { free(p); }
}
