// libnts_io.so — the reference's on-disk formats at scale (C-ABI, include/nts_io.h).
//
// Host-side loaders for inputs beyond what numpy's text readers handle in
// reasonable time or memory: the binary edge list is
// memory-mapped and read in chunks (the caller streams them to the device),
// the text feature / label / mask files are parsed in parallel straight into
// the caller's arrays with the reference's lock-step semantics
// (GNNDatum::readFeature_Label_Mask, core/ntsDataloador.hpp:999-1064).
#include "nts_io.h"

#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return NTS_IO_ERR;
}

// read-only mapping of a whole file
struct Map {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return false;
    p = static_cast<const char*>(m);
    madvise(m, n, MADV_SEQUENTIAL);
    return true;
  }
  ~Map() {
    if (p) munmap(const_cast<char*>(p), n);
    if (fd >= 0) ::close(fd);
  }
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

inline const char* skip_space(const char* s, const char* e) {
  while (s < e && is_space(*s)) ++s;
  return s;
}
inline const char* skip_token(const char* s, const char* e) {
  while (s < e && !is_space(*s)) ++s;
  return s;
}

// `>>` of a whitespace-separated token as the given type (what the
// reference's std::ifstream extraction reads)
template <typename T>
inline const char* parse(const char* s, const char* e, T& out, bool& ok) {
  s = skip_space(s, e);
  if (s >= e) {
    ok = false;
    return s;
  }
  const char* t = skip_token(s, e);
  if (*s == '+') ++s;  // from_chars takes no leading '+', istream does
  auto r = std::from_chars(s, t, out);
  ok = r.ec == std::errc() && r.ptr == t;
  return t;
}

// [begin, end) offsets of `parts` pieces of the text cut at line starts
std::vector<size_t> line_cuts(const char* p, size_t n, int parts) {
  std::vector<size_t> cut(parts + 1, n);
  cut[0] = 0;
  for (int i = 1; i < parts; ++i) {
    size_t o = std::min(std::max<size_t>(n / parts * i, 1), n);  // p[o - 1] stays in the text
    while (o < n && p[o - 1] != '\n') ++o;
    cut[i] = std::max(o, cut[i - 1]);
  }
  return cut;
}

// data lines (non-blank) of the text, in order: their start offsets
std::vector<size_t> line_starts(const char* p, size_t n, int threads) {
  const std::vector<size_t> cut = line_cuts(p, n, threads);
  std::vector<std::vector<size_t>> part(threads);
#pragma omp parallel for num_threads(threads) schedule(static, 1)
  for (int t = 0; t < threads; ++t) {
    size_t o = cut[t];
    while (o < cut[t + 1]) {
      size_t q = o;
      while (q < cut[t + 1] && p[q] != '\n') ++q;
      size_t a = o;
      while (a < q && is_space(p[a])) ++a;
      if (a < q) part[t].push_back(o);
      o = q + 1;
    }
  }
  std::vector<size_t> out;
  for (auto& v : part) out.insert(out.end(), v.begin(), v.end());
  return out;
}

}  // namespace

extern "C" {

const char* nts_io_last_error(void) { return g_err.c_str(); }

int64_t nts_io_edge_count(const char* path) {
  struct stat st;
  if (!path || stat(path, &st) != 0) return fail(std::string("cannot stat ") + (path ? path : "")), -1;
  if (st.st_size % 8 != 0) return fail(std::string(path) + ": size is not a multiple of 8 bytes"), -1;
  return (int64_t)(st.st_size / 8);
}

int nts_io_read_edges(const char* path, uint64_t first, uint64_t count, uint32_t* src,
                      uint32_t* dst) {
  if (!path || (!src && count) || (!dst && count)) return fail("NULL argument");
  Map m;
  if (!m.open(path)) return fail(std::string("cannot map ") + path);
  if (m.n % 8) return fail(std::string(path) + ": size is not a multiple of 8 bytes");
  const uint64_t E = m.n / 8;
  if (first > E || count > E - first) return fail("edge range past the end of the file");
  const uint32_t* e = reinterpret_cast<const uint32_t*>(m.p) + 2 * first;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)count; ++i) {
    src[i] = e[2 * i];
    dst[i] = e[2 * i + 1];
  }
  return NTS_IO_OK;
}

int nts_io_read_feature_label_mask(const char* feature_path, const char* label_path,
                                   const char* mask_path, uint64_t n_vertices, uint32_t F,
                                   float* features, int64_t* labels, int32_t* masks,
                                   int threads) {
  if (!feature_path || !label_path || !mask_path || !features || !labels || !masks)
    return fail("NULL argument");
  if (threads < 1) threads = 1;
  Map fm, lm, mm;
  if (!fm.open(feature_path)) return fail(std::string("cannot map ") + feature_path);
  if (!lm.open(label_path)) return fail(std::string("cannot map ") + label_path);
  if (!mm.open(mask_path)) return fail(std::string("cannot map ") + mask_path);
  // the k-th feature line pairs with the k-th label and mask lines; the
  // vertex id is the feature line's (the label/mask ids are read and dropped)
  const std::vector<size_t> fl = line_starts(fm.p, fm.n, threads);
  const std::vector<size_t> ll = line_starts(lm.p, lm.n, threads);
  const std::vector<size_t> ml = line_starts(mm.p, mm.n, threads);
  const size_t nl = fl.size();
  if (ll.size() < nl || ml.size() < nl)
    return fail("label/mask files have fewer lines than the feature file");
  int bad = 0;
  std::string bad_msg;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1024) reduction(| : bad)
  for (int64_t k = 0; k < (int64_t)nl; ++k) {
    bool ok = true;
    const char* fe = fm.p + (k + 1 < (int64_t)nl ? fl[k + 1] : fm.n);
    uint64_t id = 0;
    const char* s = parse(fm.p + fl[k], fe, id, ok);
    if (!ok || id >= n_vertices) {
      bad |= 1;
      continue;
    }
    float* row = features + id * F;
    for (uint32_t i = 0; i < F && ok; ++i) s = parse(s, fe, row[i], ok);
    if (!ok) {
      bad |= 2;
      continue;
    }
    const char* le = lm.p + (k + 1 < (int64_t)ll.size() ? ll[k + 1] : lm.n);
    uint64_t lid = 0;
    int64_t lab = 0;
    s = parse(lm.p + ll[k], le, lid, ok);
    s = parse(s, le, lab, ok);
    if (!ok) {
      bad |= 4;
      continue;
    }
    labels[id] = lab;
    const char* me = mm.p + (k + 1 < (int64_t)ml.size() ? ml[k + 1] : mm.n);
    const char* t = skip_token(skip_space(mm.p + ml[k], me), me);  // the id
    t = skip_space(t, me);
    const char* te = skip_token(t, me);
    const std::string_view msk(t, (size_t)(te - t));
    masks[id] = msk == "train" ? 0 : (msk == "eval" || msk == "val") ? 1 : msk == "test" ? 2 : 3;
  }
  if (bad & 1) return fail("feature file: bad or out-of-range vertex id");
  if (bad & 2) return fail("feature file: a line has fewer than F numbers");
  if (bad & 4) return fail("label file: bad line");
  return NTS_IO_OK;
}

}  // extern "C"
