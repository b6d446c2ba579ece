// libh3d.so: native reader of the reference's contact-matrix input files --
// scipy.sparse.save_npz archives (np.savez_compressed of indices / indptr /
// data / format / shape; reference analysis.py:94,100 and
// util/matrices.py:122-124 load them with scipy.sparse.load_npz). It replaces
// the Python zipfile + numpy parse of prepare_data with: the zip central
// directory read once, the three array members inflated by zlib on
// concurrent threads straight into the caller's buffers in the dtypes the
// union kernels take (indptr int64, indices int32, data float64), and the
// canonical-CSR check (sorted, duplicate-free rows) done while converting.
// Inflate and CRC-32 run through the system's libdeflate (libdeflate.so.0,
// loaded at run time: whole-buffer inflate ~3.5x and CRC ~6x zlib 1.2.11's
// on the bench's 40 MB data member, 133 -> 38 ms and 50 -> 8 ms measured),
// zlib when it is absent or H3D_NPZ_ZLIB=1.
// Host code only (g++, -lz, -ldl).
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "h3d.h"
#include "h3d_errors.h"

using h3derr::fail;

namespace {

uint16_t rd16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const unsigned char* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}
uint64_t rd64(const unsigned char* p) {
  return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}

struct Member {
  std::string name;
  uint16_t method = 0;
  uint32_t crc = 0;
  uint64_t csize = 0, usize = 0, local_off = 0;
};

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) fclose(f);
  }
};

bool read_at(FILE* f, uint64_t off, void* buf, size_t n) {
  if (fseeko(f, (off_t)off, SEEK_SET) != 0) return false;
  return fread(buf, 1, n, f) == n;
}

// the zip central directory (EOCD, ZIP64 EOCD when present)
int read_directory(FILE* f, std::vector<Member>* out) {
  if (fseeko(f, 0, SEEK_END) != 0) return fail(H3D_EARG, "npz: seek failed");
  const uint64_t size = (uint64_t)ftello(f);
  const uint64_t tail = size < 65557 ? size : 65557;
  std::vector<unsigned char> t(tail);
  if (!read_at(f, size - tail, t.data(), tail)) return fail(H3D_EARG, "npz: read failed");
  int64_t e = -1;
  for (int64_t i = (int64_t)tail - 22; i >= 0; --i)
    if (rd32(&t[i]) == 0x06054b50u) {
      e = i;
      break;
    }
  if (e < 0) return fail(H3D_EARG, "npz: no zip end record");
  uint64_t n_ent = rd16(&t[e + 10]), cd_size = rd32(&t[e + 12]), cd_off = rd32(&t[e + 16]);
  if ((n_ent == 0xFFFF || cd_off == 0xFFFFFFFFu) && e >= 20 &&
      rd32(&t[e - 20]) == 0x07064b50u) {  // ZIP64 locator -> ZIP64 EOCD
    unsigned char z[56];
    const uint64_t z_off = rd64(&t[e - 20 + 8]);
    if (z_off > size || size - z_off < 56 || !read_at(f, z_off, z, 56) ||
        rd32(z) != 0x06064b50u)
      return fail(H3D_EARG, "npz: bad zip64 end record");
    n_ent = rd64(z + 32);
    cd_size = rd64(z + 40);
    cd_off = rd64(z + 48);
  }
  // every size and offset read from the file is checked against the file
  // before it sizes an allocation or a read
  if (cd_off > size || cd_size > size - cd_off || n_ent > cd_size / 46)
    return fail(H3D_EARG, "npz: central directory outside the file");
  std::vector<unsigned char> cd(cd_size);
  if (!read_at(f, cd_off, cd.data(), cd_size)) return fail(H3D_EARG, "npz: read failed");
  size_t p = 0;
  for (uint64_t k = 0; k < n_ent; ++k) {
    if (p + 46 > cd.size() || rd32(&cd[p]) != 0x02014b50u)
      return fail(H3D_EARG, "npz: bad central directory");
    Member m;
    m.method = rd16(&cd[p + 10]);
    m.crc = rd32(&cd[p + 16]);
    m.csize = rd32(&cd[p + 20]);
    m.usize = rd32(&cd[p + 24]);
    const uint16_t nl = rd16(&cd[p + 28]), xl = rd16(&cd[p + 30]), cl = rd16(&cd[p + 32]);
    if (p + 46 + (size_t)nl + xl + cl > cd.size())
      return fail(H3D_EARG, "npz: central directory entry overruns the directory");
    m.local_off = rd32(&cd[p + 42]);
    m.name.assign((const char*)&cd[p + 46], nl);
    // ZIP64 extra field: the 0xFFFFFFFF fields follow in order
    size_t x = p + 46 + nl;
    const size_t xe = x + xl;
    while (x + 4 <= xe) {
      const uint16_t id = rd16(&cd[x]), len = rd16(&cd[x + 2]);
      if (x + 4 + len > xe) return fail(H3D_EARG, "npz: extra field overruns its entry");
      if (id == 0x0001) {
        size_t q = x + 4;
        const size_t qe = x + 4 + len;
        if (m.usize == 0xFFFFFFFFu && q + 8 <= qe) m.usize = rd64(&cd[q]), q += 8;
        if (m.csize == 0xFFFFFFFFu && q + 8 <= qe) m.csize = rd64(&cd[q]), q += 8;
        if (m.local_off == 0xFFFFFFFFu && q + 8 <= qe) m.local_off = rd64(&cd[q]);
      }
      x += 4 + len;
    }
    // a member lies inside the file, and deflate expands at most ~1032x
    if (m.local_off > size || m.csize > size - m.local_off ||
        (m.method == 0 && m.usize != m.csize) ||
        m.usize > m.csize * 1040 + 4096)
      return fail(H3D_EARG, "npz: member %s sizes outside the file", m.name.c_str());
    out->push_back(m);
    p += 46 + nl + xl + cl;
  }
  return 0;
}

// libdeflate's whole-buffer API (libdeflate.h of 1.0+, the symbols
// libdeflate.so.0 exports): resolved once; null pointers = use zlib
struct Deflate {
  void* (*alloc)() = nullptr;
  void (*free_d)(void*) = nullptr;
  int (*decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
  uint32_t (*crc32)(uint32_t, const void*, size_t) = nullptr;
  Deflate() {
    const char* z = std::getenv("H3D_NPZ_ZLIB");
    if (z && z[0] == '1') return;
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
    free_d = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
    decompress = (int (*)(void*, const void*, size_t, void*, size_t, size_t*))dlsym(
        h, "libdeflate_deflate_decompress");
    crc32 = (uint32_t(*)(uint32_t, const void*, size_t))dlsym(h, "libdeflate_crc32");
    if (!alloc || !free_d || !decompress || !crc32) alloc = nullptr, crc32 = nullptr;
  }
};
const Deflate& deflate_lib() {
  static const Deflate d;  // thread-safe initialisation (C++11)
  return d;
}

}  // namespace

extern "C" int h3d_npz_backend() { return deflate_lib().alloc ? 1 : 0; }

namespace {

// the zip CRC-32 of the member's bytes (zipfile raises BadZipFile on a
// mismatch; so do we)
// (zlib's table CRC runs ~0.5 GB/s: large members are split over threads
// and the pieces joined with crc32_combine)
uLong crc_range(const unsigned char* p, size_t n) {
  uLong c = crc32(0L, Z_NULL, 0);
  for (size_t o = 0; o < n; o += 1u << 30)
    c = crc32(c, p + o, (uInt)std::min<size_t>(n - o, 1u << 30));
  return c;
}

int check_crc(const Member& m, const unsigned char* b, size_t size) {
  if (const auto crc = deflate_lib().crc32) {
    if (crc(0, b, size) != m.crc)
      return fail(H3D_EARG, "npz: CRC mismatch (%s)", m.name.c_str());
    return 0;
  }
  const size_t kPiece = 4u << 20;
  const int pieces = (int)std::min<size_t>(8, (size + kPiece - 1) / kPiece);
  uLong c;
  if (pieces <= 1) {
    c = crc_range(b, size);
  } else {
    const size_t len = (size + pieces - 1) / pieces;
    std::vector<uLong> part(pieces);
    std::vector<std::thread> th;
    for (int i = 1; i < pieces; ++i)
      th.emplace_back([&, i] {
        const size_t o = i * len;
        part[i] = crc_range(b + o, std::min(len, size - o));
      });
    part[0] = crc_range(b, len);
    for (auto& t : th) t.join();
    c = part[0];
    for (int i = 1; i < pieces; ++i)
      c = crc32_combine(c, part[i], (z_off_t)std::min(len, size - i * len));
  }
  if ((uint32_t)c != m.crc) return fail(H3D_EARG, "npz: CRC mismatch (%s)", m.name.c_str());
  return 0;
}

// the member's m.usize bytes, inflated (method 8) or stored (0), into `dst`
// (the caller's buffer or member_bytes' vector), CRC-checked
int member_into(FILE* f, const Member& m, unsigned char* dst) {
  unsigned char lh[30];
  if (!read_at(f, m.local_off, lh, 30) || rd32(lh) != 0x04034b50u)
    return fail(H3D_EARG, "npz: bad local header (%s)", m.name.c_str());
  const uint64_t data_off = m.local_off + 30 + rd16(lh + 26) + rd16(lh + 28);
  if (m.method == 0) {
    if (m.usize && !read_at(f, data_off, dst, m.usize))
      return fail(H3D_EARG, "npz: read failed (%s)", m.name.c_str());
    return check_crc(m, dst, m.usize);
  }
  if (m.method != 8) return fail(H3D_EARG, "npz: compression method %d", (int)m.method);
  std::vector<unsigned char> comp(m.csize);
  if (m.csize && !read_at(f, data_off, comp.data(), m.csize))
    return fail(H3D_EARG, "npz: read failed (%s)", m.name.c_str());
  const Deflate& L = deflate_lib();
  if (L.alloc) {
    void* d = L.alloc();
    if (!d) return fail(H3D_ENOMEM, "npz: libdeflate decompressor");
    size_t got = 0;
    const int r = L.decompress(d, comp.data(), comp.size(), dst, m.usize, &got);
    L.free_d(d);
    if (r != 0 || got != m.usize)
      return fail(H3D_EARG, "npz: inflate failed (%s)", m.name.c_str());
    return check_crc(m, dst, m.usize);
  }
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) return fail(H3D_EARG, "npz: inflateInit failed");
  // the sizes may exceed uInt: feed and drain in chunks
  uint64_t in_done = 0, out_done = 0;
  int rc = Z_OK;
  while (rc != Z_STREAM_END) {
    if (zs.avail_in == 0 && in_done < m.csize) {
      const uint64_t c = std::min<uint64_t>(m.csize - in_done, 1u << 30);
      zs.next_in = comp.data() + in_done;
      zs.avail_in = (uInt)c;
      in_done += c;
    }
    if (zs.avail_out == 0) {
      const uint64_t c = std::min<uint64_t>(m.usize - out_done, 1u << 30);
      if (c == 0) break;
      zs.next_out = dst + out_done;
      zs.avail_out = (uInt)c;
      out_done += c;
    }
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) break;
  }
  inflateEnd(&zs);
  if (rc != Z_STREAM_END || zs.total_out != m.usize)
    return fail(H3D_EARG, "npz: inflate failed (%s)", m.name.c_str());
  return check_crc(m, dst, m.usize);
}

int member_bytes(FILE* f, const Member& m, std::vector<unsigned char>* out) {
  out->resize(m.usize);
  return member_into(f, m, out->data());
}

// the first `n` uncompressed bytes of the member (headers: no full inflate)
int member_head(FILE* f, const Member& m, size_t n, std::vector<unsigned char>* out) {
  unsigned char lh[30];
  if (!read_at(f, m.local_off, lh, 30) || rd32(lh) != 0x04034b50u)
    return fail(H3D_EARG, "npz: bad local header (%s)", m.name.c_str());
  const uint64_t data_off = m.local_off + 30 + rd16(lh + 26) + rd16(lh + 28);
  n = (size_t)std::min<uint64_t>(n, m.usize);
  if (m.method == 0) {
    out->resize(n);
    if (n && !read_at(f, data_off, out->data(), n))
      return fail(H3D_EARG, "npz: read failed (%s)", m.name.c_str());
    return 0;
  }
  if (m.method != 8) return fail(H3D_EARG, "npz: compression method %d", (int)m.method);
  const size_t cn = (size_t)std::min<uint64_t>(m.csize, n + 4096);
  std::vector<unsigned char> comp(cn);
  if (cn && !read_at(f, data_off, comp.data(), cn))
    return fail(H3D_EARG, "npz: read failed (%s)", m.name.c_str());
  out->resize(n);
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) return fail(H3D_EARG, "npz: inflateInit failed");
  zs.next_in = comp.data();
  zs.avail_in = (uInt)cn;
  zs.next_out = out->data();
  zs.avail_out = (uInt)n;
  int rc = Z_OK;
  while (zs.avail_out && rc == Z_OK) rc = inflate(&zs, Z_SYNC_FLUSH);
  inflateEnd(&zs);
  if (rc != Z_OK && rc != Z_STREAM_END && rc != Z_BUF_ERROR)
    return fail(H3D_EARG, "npz: inflate failed (%s)", m.name.c_str());
  out->resize(zs.total_out);
  return 0;
}

// .npy header: dtype kind / size, C order, shape
struct Npy {
  char kind = 0;  // 'i', 'u', 'f', 'b', 'U', 'S'
  int itemsize = 0;
  bool little = true;
  std::vector<int64_t> shape;
  size_t data_off = 0;
};

int parse_npy(const std::vector<unsigned char>& b, Npy* h, const char* what) {
  if (b.size() < 10 || std::memcmp(b.data(), "\x93NUMPY", 6) != 0)
    return fail(H3D_EARG, "npz: %s is not a .npy", what);
  const int major = b[6];
  size_t hl, ho;
  if (major == 1) {
    hl = rd16(&b[8]);
    ho = 10;
  } else {
    hl = rd32(&b[8]);
    ho = 12;
  }
  if (ho + hl > b.size()) return fail(H3D_EARG, "npz: %s header truncated", what);
  const std::string s((const char*)&b[ho], hl);
  h->data_off = ho + hl;
  const size_t d = s.find("'descr'");
  const size_t q1 = s.find('\'', s.find(':', d) + 1);
  const size_t q2 = s.find('\'', q1 + 1);
  if (d == std::string::npos || q1 == std::string::npos || q2 == std::string::npos)
    return fail(H3D_EARG, "npz: %s has no dtype", what);
  const std::string descr = s.substr(q1 + 1, q2 - q1 - 1);  // e.g. <i4, |b1, <U3
  if (descr.size() < 3) return fail(H3D_EARG, "npz: %s dtype %s", what, descr.c_str());
  h->little = descr[0] != '>';
  h->kind = descr[1];
  h->itemsize = std::atoi(descr.c_str() + 2);
  if (s.find("'fortran_order': True") != std::string::npos)
    return fail(H3D_EARG, "npz: %s is Fortran-ordered", what);
  const size_t sp = s.find('(', s.find("'shape'"));
  const size_t se = s.find(')', sp);
  size_t i = sp + 1;
  while (i < se) {
    while (i < se && (s[i] == ' ' || s[i] == ',')) ++i;
    if (i >= se) break;
    h->shape.push_back(std::atoll(s.c_str() + i));
    while (i < se && s[i] != ',') ++i;
  }
  return 0;
}

int64_t npy_count(const Npy& h) {
  int64_t n = 1;
  for (int64_t v : h.shape) n *= v;
  return n;
}

// element k of an integer / float .npy payload as T
template <typename T>
bool npy_convert(const std::vector<unsigned char>& b, const Npy& h, T* out, int64_t n) {
  if (!h.little && h.itemsize > 1) return false;
  if ((int64_t)(b.size() - h.data_off) < n * h.itemsize) return false;
  const unsigned char* p = b.data() + h.data_off;
#define H3D_CONV(CT)                               \
  for (int64_t k = 0; k < n; ++k) {                \
    CT v;                                          \
    std::memcpy(&v, p + k * sizeof(CT), sizeof(CT)); \
    out[k] = (T)v;                                 \
  }                                                \
  return true
  if (h.kind == 'f' && h.itemsize == 8) { H3D_CONV(double); }
  if (h.kind == 'f' && h.itemsize == 4) { H3D_CONV(float); }
  if (h.kind == 'i' && h.itemsize == 8) { H3D_CONV(int64_t); }
  if (h.kind == 'i' && h.itemsize == 4) { H3D_CONV(int32_t); }
  if (h.kind == 'i' && h.itemsize == 2) { H3D_CONV(int16_t); }
  if (h.kind == 'i' && h.itemsize == 1) { H3D_CONV(int8_t); }
  if (h.kind == 'u' && h.itemsize == 8) { H3D_CONV(uint64_t); }
  if (h.kind == 'u' && h.itemsize == 4) { H3D_CONV(uint32_t); }
  if (h.kind == 'u' && h.itemsize == 2) { H3D_CONV(uint16_t); }
  if ((h.kind == 'u' || h.kind == 'b') && h.itemsize == 1) { H3D_CONV(uint8_t); }
#undef H3D_CONV
  return false;
}

struct Archive {
  File file;
  std::vector<Member> members;
  const Member* get(const char* name) const {
    for (const Member& m : members)
      if (m.name == name) return &m;
    return nullptr;
  }
};

int open_archive(const char* path, Archive* a) {
  a->file.f = fopen(path, "rb");
  if (!a->file.f) return fail(H3D_EARG, "npz: cannot open %s", path);
  return read_directory(a->file.f, &a->members);
}

int small_member(Archive& a, const char* name, std::vector<unsigned char>* bytes, Npy* h) {
  const Member* m = a.get(name);
  if (!m) return fail(H3D_EARG, "npz: no %s member", name);
  if (int rc = member_bytes(a.file.f, *m, bytes)) return rc;
  return parse_npy(*bytes, h, name);
}

}  // namespace

namespace {
int csr_info(const char* path, int64_t* n_rows, int64_t* n_cols, int64_t* nnz);
int csr_read(const char* path, int64_t n_rows, int64_t nnz, int64_t* indptr,
             int32_t* indices, double* data, int64_t slack, int* canonical);
}  // namespace

extern "C" {

// the entry points turn any exception (a bad_alloc sized by a corrupt
// archive) into an error code: nothing may unwind through the C ABI
int h3d_npz_csr_info(const char* path, int64_t* n_rows, int64_t* n_cols, int64_t* nnz) {
  try {
    return csr_info(path, n_rows, n_cols, nnz);
  } catch (const std::exception& e) {
    return fail(H3D_ENOMEM, "npz: %s", e.what());
  }
}

int h3d_npz_csr_read(const char* path, int64_t n_rows, int64_t nnz, int64_t* indptr,
                     int32_t* indices, double* data, int* canonical) {
  try {
    return csr_read(path, n_rows, nnz, indptr, indices, data, 0, canonical);
  } catch (const std::exception& e) {
    return fail(H3D_ENOMEM, "npz: %s", e.what());
  }
}

int h3d_npz_csr_read_slack(const char* path, int64_t n_rows, int64_t nnz, int64_t* indptr,
                           int32_t* indices, double* data, int64_t slack, int* canonical) {
  try {
    return csr_read(path, n_rows, nnz, indptr, indices, data, slack < 0 ? 0 : slack,
                    canonical);
  } catch (const std::exception& e) {
    return fail(H3D_ENOMEM, "npz: %s", e.what());
  }
}

// One number per line, as np.loadtxt reads a one-column file (load_bias,
// core.py:35-60, the replicates' bias vectors): blank lines and '#' comments
// skipped, each value by strtod (correctly rounded, as numpy's own parser).
// Anything else -- two tokens on a line, a hex float, trailing characters --
// is H3D_EINPUT, and the caller reads the file with np.loadtxt instead.
// Host only, no GIL: prepare_data's reader thread calls it while the main
// thread drives the device.
int h3d_read_text_column(const char* path, double* out, int64_t cap, int64_t* n) {
  if (!path || !n || (cap > 0 && !out)) return fail(H3D_EARG, "null argument");
  *n = 0;
  FILE* fh = std::fopen(path, "rb");
  if (!fh) return fail(H3D_EARG, "text column: cannot open %s", path);
  std::vector<char> text;
  try {
    char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof(buf), fh)) > 0) text.insert(text.end(), buf, buf + got);
  } catch (const std::exception& e) {
    std::fclose(fh);
    return fail(H3D_ENOMEM, "text column: %s", e.what());
  }
  std::fclose(fh);
  text.push_back('\0');
  const char* q = text.data();
  const char* end = q + text.size() - 1;
  int64_t k = 0;
  while (q < end) {
    const char* eol = static_cast<const char*>(std::memchr(q, '\n', end - q));
    if (!eol) eol = end;
    const char* hash = static_cast<const char*>(std::memchr(q, '#', eol - q));
    const char* le = hash ? hash : eol;
    const char* a = q;
    while (a < le && std::isspace((unsigned char)*a)) ++a;
    const char* b = le;
    while (b > a && std::isspace((unsigned char)b[-1])) --b;
    if (a < b) {
      for (const char* c = a; c < b; ++c)
        if (std::isspace((unsigned char)*c) || *c == 'x' || *c == 'X')
          return fail(H3D_EINPUT, "text column: %s line %lld is not one number", path,
                      (long long)(k + 1));
      char* stop = nullptr;
      const double v = std::strtod(a, &stop);
      if (stop != b) return fail(H3D_EINPUT, "text column: %s: not a number", path);
      if (k >= cap) return fail(H3D_EARG, "text column: %s has more than %lld values", path,
                                (long long)cap);
      out[k++] = v;
    }
    q = eol + 1;
  }
  *n = k;
  return 0;
}

}  // extern "C"

namespace {

int csr_info(const char* path, int64_t* n_rows, int64_t* n_cols, int64_t* nnz) {
  if (!path || !n_rows || !n_cols || !nnz) return fail(H3D_EARG, "null argument");
  Archive a;
  if (int rc = open_archive(path, &a)) return rc;
  std::vector<unsigned char> b;
  Npy h;
  if (int rc = small_member(a, "format.npy", &b, &h)) return rc;
  const std::string fmt((const char*)b.data() + h.data_off, b.size() - h.data_off);
  // format is a 0-d string array: 'csr' as UTF-32 ('<U3') or bytes ('|S3')
  const bool csr = (h.kind == 'U' && b.size() >= h.data_off + 12 && b[h.data_off] == 'c' &&
                    b[h.data_off + 4] == 's' && b[h.data_off + 8] == 'r') ||
                   (h.kind == 'S' && fmt.compare(0, 3, "csr") == 0);
  if (!csr) return fail(H3D_EARG, "npz: %s is not a CSR matrix", path);
  if (int rc = small_member(a, "shape.npy", &b, &h)) return rc;
  int64_t shp[2];
  if (npy_count(h) != 2 || !npy_convert<int64_t>(b, h, shp, 2))
    return fail(H3D_EARG, "npz: bad shape member");
  const Member* md = a.get("data.npy");
  if (!md) return fail(H3D_EARG, "npz: no data member");
  // the data member's header: inflate its first bytes only
  std::vector<unsigned char> head;
  if (int rc = member_head(a.file.f, *md, 4096, &head)) return rc;
  Npy hd;
  if (int rc = parse_npy(head, &hd, "data.npy")) return rc;
  if (shp[0] < 0 || shp[1] < 0 || shp[0] > ((int64_t)1 << 40))
    return fail(H3D_EARG, "npz: bad shape");
  for (int64_t v : hd.shape)
    if (v < 0) return fail(H3D_EARG, "npz: bad data shape");
  *n_rows = shp[0];
  *n_cols = shp[1];
  *nnz = npy_count(hd);
  return 0;
}

// the three arrays into caller buffers (n_rows + 1, nnz, nnz); *canonical =
// 1 when every row's column indices are strictly increasing (sorted, no
// duplicates: what the union kernels take as is). With `slack` writable
// bytes before `indices` and `data`, a member already in the target dtype
// (little-endian int32 / float64) whose .npy header fits the slack is
// inflated in place -- header into the slack, payload straight into the
// caller's array -- instead of through a scratch copy (the bench's 40 MB data
// member: no 40 MB allocation, page-fault pass or copy).
int csr_read(const char* path, int64_t n_rows, int64_t nnz, int64_t* indptr,
             int32_t* indices, double* data, int64_t slack, int* canonical) {
  if (!path || !indptr || (nnz && (!indices || !data)) || !canonical)
    return fail(H3D_EARG, "null argument");
  if (n_rows < 0 || nnz < 0) return fail(H3D_EARG, "npz: n_rows / nnz");
  Archive a;
  if (int rc = open_archive(path, &a)) return rc;
  const char* names[3] = {"indptr.npy", "indices.npy", "data.npy"};
  int rcs[3] = {0, 0, 0};
  std::string errs[3];
  auto work = [&](int j) {
    const Member* m = a.get(names[j]);
    if (!m) {
      rcs[j] = fail(H3D_EARG, "npz: no %s member", names[j]);
      errs[j] = h3derr::last();
      return;
    }
    // each thread reads through its own FILE (one stream is not shareable);
    // an exception (bad_alloc) must not leave the thread
    try {
    File own;
    own.f = fopen(path, "rb");
    if (own.f && j > 0 && slack > 0 && nnz > 0) {
      // in place when the payload has the target's width: int32 indices;
      // 8-byte data (float64 as is, int64 / uint64 counts converted to
      // float64 in place afterwards, element k onto itself)
      std::vector<unsigned char> head;
      Npy hh;
      const int itemsize = j == 1 ? 4 : 8;
      if (!member_head(own.f, *m, 1024, &head) && !parse_npy(head, &hh, names[j]) &&
          (j == 1 ? hh.kind == 'i' : (hh.kind == 'f' || hh.kind == 'i' || hh.kind == 'u')) &&
          hh.itemsize == itemsize && hh.little && (int64_t)hh.data_off <= slack &&
          npy_count(hh) == nnz && m->usize == hh.data_off + (uint64_t)nnz * itemsize) {
        unsigned char* dst = (j == 1 ? (unsigned char*)indices : (unsigned char*)data);
        rcs[j] = member_into(own.f, *m, dst - hh.data_off);
        if (rcs[j]) {
          errs[j] = h3derr::last();
        } else if (j == 2 && hh.kind == 'i') {
          for (int64_t k = 0; k < nnz; ++k) {
            int64_t v;
            std::memcpy(&v, data + k, 8);
            data[k] = (double)v;
          }
        } else if (j == 2 && hh.kind == 'u') {
          for (int64_t k = 0; k < nnz; ++k) {
            uint64_t v;
            std::memcpy(&v, data + k, 8);
            data[k] = (double)v;
          }
        }
        return;
      }
    }
    std::vector<unsigned char> b;
    Npy h;
    int rc = own.f ? member_bytes(own.f, *m, &b) : fail(H3D_EARG, "npz: reopen failed");
    if (!rc) rc = parse_npy(b, &h, names[j]);
    const int64_t want = j == 0 ? n_rows + 1 : nnz;
    if (!rc && npy_count(h) != want)
      rc = fail(H3D_EARG, "npz: %s has %lld entries, expected %lld", names[j],
                (long long)npy_count(h), (long long)want);
    bool ok = true;
    if (!rc) {
      if (j == 0) ok = npy_convert<int64_t>(b, h, indptr, want);
      else if (j == 1) ok = npy_convert<int32_t>(b, h, indices, want);
      else ok = npy_convert<double>(b, h, data, want);
      if (!ok) rc = fail(H3D_EARG, "npz: %s dtype %c%d not supported", names[j], h.kind, h.itemsize);
    }
    rcs[j] = rc;
    if (rc) errs[j] = h3derr::last();
    } catch (const std::exception& ex) {
      rcs[j] = H3D_ENOMEM;
      errs[j] = std::string("npz: ") + ex.what();
    }
  };
  std::thread t1(work, 1), t2(work, 2);
  work(0);
  t1.join();
  t2.join();
  for (int j = 0; j < 3; ++j)
    if (rcs[j]) return fail(rcs[j], "%s", errs[j].c_str());
  if (indptr[0] != 0 || indptr[n_rows] != nnz) return fail(H3D_EARG, "npz: bad indptr");
  // the whole indptr before any row is scanned: 0 <= indptr[r] <=
  // indptr[r + 1] <= nnz, so no row reads past the indices
  for (int64_t r = 0; r < n_rows; ++r)
    if (indptr[r + 1] < indptr[r] || indptr[r + 1] > nnz)
      return fail(H3D_EARG, "npz: bad indptr (row %lld)", (long long)r);
  int canon = 1;
  for (int64_t r = 0; r < n_rows && canon; ++r) {
    for (int64_t k = indptr[r] + 1; k < indptr[r + 1]; ++k)
      if (indices[k] <= indices[k - 1]) {
        canon = 0;
        break;
      }
  }
  *canonical = canon;
  return 0;
}

}  // namespace
