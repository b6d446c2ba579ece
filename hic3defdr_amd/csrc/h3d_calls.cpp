// Host side of the differential-call steps downstream of the q-values
// (threshold -> classify -> collect, reference analysis.py:366-572):
// clustering of thresholded pixels and the text forms of the clusters.
//
// h3d_find_clusters restates hic3defdr/util/clusters.py:73-97 find_clusters
// with its DirectedDisjointSet (:15-70) event for event, so the clusters come
// out as the same pixel sets AND in the same order as the reference's
// get_groups() (a dict of group leaders in creation order, where a merge keeps
// the larger group -- the centre's group on a tie -- and drops the other
// leader). The work is a sequence of dependent union steps over the pixel
// list, which is why it runs on the host; the per-pixel statistics that
// produce the q-values are the GPU's.
#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "h3d.h"
#include "h3d_errors.h"

namespace h3derr {

namespace {
thread_local std::string g_err;
}

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

const char* last() { return g_err.c_str(); }

}  // namespace h3derr

namespace {

using h3derr::fail;

inline uint64_t pixel_key(int64_t r, int64_t c) {
  return ((uint64_t)(uint32_t)r << 32) | (uint32_t)c;
}

// The DirectedDisjointSet over pixel nodes. Group membership is an intrusive
// singly linked list per leader, so a merge relabels the absorbed (smaller)
// group exactly like the reference's `for k in groupb: leader[k] = leadera`.
struct Dds {
  std::vector<int32_t> leader, next, tail, size;
  std::vector<int64_t> born;  // creation stamp of a group's leader (dict order)
  int64_t stamp = 0;

  explicit Dds(size_t n)
      : leader(n, -1), next(n, -1), tail(n, -1), size(n, 0), born(n, -1) {}

  // clusters.py:34-66 (add a -> b); b < 0 = a pixel outside the point set
  void add(int32_t a, int32_t b) {
    int32_t la = leader[a];
    const int32_t lb = b >= 0 ? leader[b] : -1;
    if (la >= 0) {
      if (lb < 0 || la == lb) return;
      int32_t keep = la, drop = lb;
      if (size[la] < size[lb]) {
        keep = lb;
        drop = la;
      }
      for (int32_t k = drop; k >= 0; k = next[k]) leader[k] = keep;
      next[tail[keep]] = drop;
      tail[keep] = tail[drop];
      size[keep] += size[drop];
      size[drop] = 0;
      born[drop] = -1;
      return;
    }
    if (lb >= 0) {  // a joins b's group
      leader[a] = lb;
      next[tail[lb]] = a;
      tail[lb] = a;
      size[lb] += 1;
    } else {  // new group {a}
      leader[a] = a;
      tail[a] = a;
      size[a] = 1;
      born[a] = stamp++;
    }
  }
};

}  // namespace

extern "C" {

int h3d_find_clusters(const int64_t* row, const int64_t* col, int64_t n,
                      int connectivity, int64_t* label, int64_t* n_clusters) {
  if (n < 0 || !n_clusters || (n > 0 && (!row || !col || !label)))
    return fail(H3D_EARG, "find_clusters: null argument");
  if (n > 0x7ffffffeLL) return fail(H3D_EARG, "find_clusters: too many pixels");
  // scipy generate_binary_structure(2, connectivity) -> np.where order
  // (row-major over the 3x3 neighbourhood, |dr| + |dc| <= connectivity)
  int sr[9], sc[9], ns = 0;
  for (int dr = -1; dr <= 1; ++dr)
    for (int dc = -1; dc <= 1; ++dc) {
      const int m = (dr < 0 ? -dr : dr) + (dc < 0 ? -dc : dc);
      if (m <= (connectivity < 0 ? 0 : connectivity)) {
        sr[ns] = dr;
        sc[ns] = dc;
        ++ns;
      }
    }
  // pixel -> node (first occurrence); duplicate COO entries share a node
  std::unordered_map<uint64_t, int32_t> node_of;
  node_of.reserve((size_t)n * 2 + 1);
  std::vector<int32_t> node(n);
  for (int64_t i = 0; i < n; ++i) {
    if (row[i] < 0 || col[i] < 0 || row[i] > 0x7fffffff || col[i] > 0x7fffffff)
      return fail(H3D_EARG, "find_clusters: pixel (%lld, %lld) out of range",
                  (long long)row[i], (long long)col[i]);
    auto it = node_of.emplace(pixel_key(row[i], col[i]), (int32_t)node_of.size());
    node[i] = it.first->second;
  }
  Dds dds(node_of.size());
  for (int64_t i = 0; i < n; ++i) {
    for (int s = 0; s < ns; ++s) {
      const int64_t r = row[i] + sr[s], c = col[i] + sc[s];
      int32_t b = -1;
      if (r >= 0 && c >= 0) {
        auto it = node_of.find(pixel_key(r, c));
        if (it != node_of.end()) b = it->second;
      }
      dds.add(node[i], b);
    }
  }
  // surviving leaders in creation order = get_groups() order
  const size_t nn = node_of.size();
  std::vector<int64_t> rank_of(nn, -1);
  std::vector<std::pair<int64_t, int32_t>> alive;
  for (size_t k = 0; k < nn; ++k)
    if (dds.born[k] >= 0 && dds.leader[k] == (int32_t)k)
      alive.emplace_back(dds.born[k], (int32_t)k);
  std::sort(alive.begin(), alive.end());
  for (size_t j = 0; j < alive.size(); ++j) rank_of[alive[j].second] = (int64_t)j;
  for (int64_t i = 0; i < n; ++i) label[i] = rank_of[dds.leader[node[i]]];
  *n_clusters = (int64_t)alive.size();
  return 0;
}

// Text of clusters as the reference's JSON / TSV write them
// (clusters.py:129-130 json.dump of [[i, j], ...]; cluster_table.py:67 str of
// a list of [i, j] lists): cluster k = pixels order[starts[k] .. starts[k+1])
// -> "[[i, j], [i, j]]". Writes the concatenated strings to buf (capacity cap;
// buf may be NULL to size) and their end offsets to ends (n_clusters, may be
// NULL); *len = total bytes.
int h3d_format_clusters(const int64_t* row, const int64_t* col,
                        const int64_t* order, const int64_t* starts,
                        int64_t n_clusters, char* buf, int64_t cap,
                        int64_t* ends, int64_t* len) {
  if (n_clusters < 0 || !len || (n_clusters > 0 && (!row || !col || !order || !starts)))
    return fail(H3D_EARG, "format_clusters: null argument");
  int64_t pos = 0;
  char tmp[64];
  auto put = [&](const char* s, int64_t m) {
    if (buf && pos + m <= cap) std::memcpy(buf + pos, s, (size_t)m);
    pos += m;
  };
  for (int64_t k = 0; k < n_clusters; ++k) {
    put("[", 1);
    for (int64_t j = starts[k]; j < starts[k + 1]; ++j) {
      const int64_t i = order[j];
      const int m = std::snprintf(tmp, sizeof(tmp), "%s[%lld, %lld]",
                                  j > starts[k] ? ", " : "", (long long)row[i],
                                  (long long)col[i]);
      put(tmp, m);
    }
    put("]", 1);
    if (ends) ends[k] = pos;
  }
  *len = pos;
  if (buf && pos > cap) return fail(H3D_EARG, "format_clusters: buffer too small");
  return 0;
}

}  // extern "C"
