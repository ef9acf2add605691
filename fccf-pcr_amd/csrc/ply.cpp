// ply.cpp — PLY reader/writer for the CLI surface of FCCF.cpp:1655-1665
// (pcl::io::loadPLYFile<PointXYZ>): ascii, binary_little_endian and
// binary_big_endian vertex elements; x, y, z mapped by name; every other property
// (and every other element) is skipped by size.
//
// Value conversion follows PCL 1.10's ply_parser: a binary value is read in its
// declared type and converted to the float field; an ascii token is converted with
// the type's own parser (float tokens correctly rounded straight to float, as
// libstdc++'s istream >> float does under boost::lexical_cast; double tokens to
// double, then narrowed), and a token that does not parse becomes a quiet NaN
// (ply_parser's bad_lexical_cast branch) instead of failing the load.
//
// The file is mapped once; binary rows of fixed size are addressed directly, other
// layouts (ascii, list properties in the vertex element) through a row index built
// in parallel.  decode() converts any row range, so the streaming ingest
// (ingest.cpp) converts chunks on several threads while earlier chunks upload.
#include "ply.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <sstream>
#include <thread>

#include "../../include/fccf.h"

namespace fccf {
namespace ply {
namespace {

int type_size(const std::string& t) {
  if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
  if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
  if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
  if (t == "double" || t == "float64") return 8;
  return 0;
}
bool is_float(const std::string& t) { return t == "float" || t == "float32"; }
bool is_double(const std::string& t) { return t == "double" || t == "float64"; }
bool is_signed_int(const std::string& t) {
  return t == "char" || t == "int8" || t == "short" || t == "int16" || t == "int" || t == "int32";
}

bool host_little() {
  const uint16_t x = 1;
  return *(const uint8_t*)&x == 1;
}

// one binary value of type t at p, converted to float (PointXYZ's field type)
float bin_value(const unsigned char* p, const std::string& t, bool swap) {
  unsigned char b[8];
  const int s = type_size(t);
  for (int i = 0; i < s; ++i) b[i] = swap ? p[s - 1 - i] : p[i];
  if (t == "char" || t == "int8") return (float)*(int8_t*)b;
  if (t == "uchar" || t == "uint8") return (float)*(uint8_t*)b;
  if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); return (float)v; }
  if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); return (float)v; }
  if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); return (float)v; }
  if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); return (float)v; }
  if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); return v; }
  double v;
  std::memcpy(&v, b, 8);
  return (float)v;
}
// A list count: -1 (rejected) unless it is a whole number in [0, 2^31) -- a count
// from the file is never converted to an integer it does not fit.
int64_t count_of(float v) { return (v >= 0.f && v < 2147483648.f) ? (int64_t)v : -1; }
int64_t bin_count(const unsigned char* p, const std::string& t, bool swap) { return count_of(bin_value(p, t, swap)); }

constexpr int64_t MAX_COUNT = 2147483647;  // element counts beyond int32 are rejected (PCL indexes with int)

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r'; }

// the next whitespace-separated token of [p, e) (a row); empty at the end of the row
const char* next_token(const char*& p, const char* e, size_t& len) {
  while (p < e && is_space(*p)) ++p;
  const char* s = p;
  while (p < e && !is_space(*p)) ++p;
  len = (size_t)(p - s);
  return s;
}

// an ascii token converted as ply_parser does (see the file comment)
float ascii_value(const char* s, size_t len, const std::string& t) {
  const float qnan = std::numeric_limits<float>::quiet_NaN();
  if (!len) return qnan;
  const char* e = s + len;
  if (*s == '+') ++s;  // accepted by the stream parsers, not by from_chars
  if (is_float(t)) {
    float v;
    const auto r = std::from_chars(s, e, v);
    return (r.ec == std::errc() && r.ptr == e) ? v : qnan;
  }
  if (is_double(t)) {
    double v;
    const auto r = std::from_chars(s, e, v);
    return (r.ec == std::errc() && r.ptr == e) ? (float)v : qnan;
  }
  if (is_signed_int(t)) {
    long long v;
    const auto r = std::from_chars(s, e, v);
    return (r.ec == std::errc() && r.ptr == e) ? (float)v : qnan;
  }
  unsigned long long v;
  const auto r = std::from_chars(s, e, v);
  return (r.ec == std::errc() && r.ptr == e) ? (float)v : qnan;
}

// one header line [p, nl) split into words
std::vector<std::string> words(const char* p, const char* e) {
  std::vector<std::string> w;
  std::istringstream ss(std::string(p, e));
  std::string x;
  while (ss >> x) w.push_back(x);
  return w;
}

// end of the row starting at p (its newline, or the end of the data)
const char* row_end(const char* p, const char* end) {
  const void* q = std::memchr(p, '\n', (size_t)(end - p));
  return q ? (const char*)q : end;
}

// Starts of the next `n` ascii rows from byte `from`, found by `threads` threads:
// each thread counts the newlines of its byte range, and the ranges' prefix gives
// the global index of each row that starts inside a range.  Returns the offset just
// past the n-th row, or (size_t)-1 if the data holds fewer rows.
size_t index_rows(const char* data, size_t size, size_t from, int64_t n, std::vector<size_t>* starts, int threads) {
  if (starts) starts->assign((size_t)n, 0);
  if (n == 0) return from;
  const size_t len = size - from;
  const int T = std::max(1, std::min(threads, (int)(len >> 20) + 1));
  std::vector<int64_t> cnt(T + 1, 0);
  auto lo = [&](int t) { return from + len * (size_t)t / (size_t)T; };
  auto count = [&](int t) {
    int64_t c = 0;
    const char* p = data + lo(t);
    const char* e = data + lo(t + 1);
    while (p < e) {
      const void* q = std::memchr(p, '\n', (size_t)(e - p));
      if (!q) break;
      ++c;
      p = (const char*)q + 1;
    }
    cnt[t + 1] = c;
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(count, t);
    count(0);
    for (auto& x : th) x.join();
  }
  for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
  // row k (0-based) starts after the k-th newline of the region (row 0 at `from`)
  auto fill = [&](int t) {
    int64_t k = cnt[t];  // rows whose start lies beyond range t's first newline
    const char* p = data + lo(t);
    const char* e = data + lo(t + 1);
    if (t == 0 && starts) (*starts)[0] = from;
    while (p < e && k + 1 < n) {
      const void* q = std::memchr(p, '\n', (size_t)(e - p));
      if (!q) break;
      p = (const char*)q + 1;
      ++k;
      if (starts) (*starts)[(size_t)k] = (size_t)(p - data);
    }
  };
  if (cnt[T] < n - 1) return (size_t)-1;  // fewer than n row starts
  if (starts) {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(fill, t);
    fill(0);
    for (auto& x : th) x.join();
  }
  // the end of row n-1: its newline (or the end of the data)
  size_t last = from;
  if (starts) last = (*starts)[(size_t)n - 1];
  else {
    int64_t k = 0;
    const char* p = data + from;
    while (k < n - 1) {
      p = row_end(p, data + size) + 1;
      ++k;
    }
    last = (size_t)(p - data);
  }
  const char* e = row_end(data + last, data + size);
  return (size_t)(e - data) + (e < data + size ? 1 : 0);
}

}  // namespace

File::~File() {
  if (data && data != (const char*)MAP_FAILED) munmap((void*)data, size);
  if (fd >= 0) ::close(fd);
}

int open(const char* path, File& f, int threads) {
  f.fd = ::open(path, O_RDONLY);
  if (f.fd < 0) return FCCF_E_IO;
  struct stat st;
  if (fstat(f.fd, &st) != 0 || st.st_size < 4) return FCCF_E_IO;
  f.size = (size_t)st.st_size;
  void* m = mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, f.fd, 0);
  if (m == MAP_FAILED) return FCCF_E_IO;
  f.data = (const char*)m;
  (void)madvise(m, f.size, MADV_SEQUENTIAL);
  const char* p = f.data;
  const char* end = f.data + f.size;
  // header
  std::string format;
  bool first = true, done = false;
  while (p < end) {
    const char* e = row_end(p, end);
    std::vector<std::string> w = words(p, e);
    p = e < end ? e + 1 : end;
    if (first) {
      if (w.empty() || w[0] != "ply") return FCCF_E_IO;
      first = false;
      continue;
    }
    if (w.empty()) continue;
    if (w[0] == "format" && w.size() > 1) format = w[1];
    else if (w[0] == "element" && w.size() > 2) {
      Elem el;
      el.name = w[1];
      // a count is a plain decimal number of at most int32 range: no wrap-around of the
      // size checks below (rec * count, 12 * count) for any header
      const std::string& cs = w[2];
      if (cs.empty() || cs.size() > 10 || cs.find_first_not_of("0123456789") != std::string::npos) return FCCF_E_IO;
      el.count = std::atoll(cs.c_str());
      if (el.count < 0 || el.count > MAX_COUNT) return FCCF_E_IO;
      f.elems.push_back(el);
    } else if (w[0] == "property") {
      if (f.elems.empty() || w.size() < 3) return FCCF_E_IO;
      Prop pr;
      if (w[1] == "list") {
        if (w.size() < 5) return FCCF_E_IO;
        pr.is_list = true;
        pr.count_type = w[2];
        pr.type = w[3];
        pr.name = w[4];
        pr.csize = type_size(pr.count_type);
        if (!pr.csize) return FCCF_E_IO;
      } else {
        pr.type = w[1];
        pr.name = w[2];
      }
      pr.size = type_size(pr.type);
      if (!pr.size) return FCCF_E_IO;
      f.elems.back().props.push_back(pr);
    } else if (w[0] == "end_header") {
      done = true;
      break;
    }
  }
  if (!done) return FCCF_E_IO;
  if (format == "ascii") f.fmt = File::ASCII;
  else if (format == "binary_little_endian") f.fmt = File::LE;
  else if (format == "binary_big_endian") f.fmt = File::BE;
  else return FCCF_E_IO;
  for (size_t i = 0; i < f.elems.size(); ++i)
    if (f.elems[i].name == "vertex") f.vi = (int)i;
  if (f.vi < 0) return FCCF_E_IO;
  const Elem& V = f.elems[(size_t)f.vi];
  for (size_t j = 0; j < V.props.size(); ++j)
    for (int a = 0; a < 3; ++a)
      if (!V.props[j].is_list && V.props[j].name == std::string(1, (char)('x' + a))) f.xyz[a] = (int)j;
  if (f.xyz[0] < 0 || f.xyz[1] < 0 || f.xyz[2] < 0) return FCCF_E_IO;
  f.n = V.count;
  size_t body = (size_t)(p - f.data);
  const bool swap = (f.fmt == File::LE && !host_little()) || (f.fmt == File::BE && host_little());
  if (f.fmt == File::ASCII) {
    // skip the rows of the elements before the vertex element, then index its rows
    for (int i = 0; i < f.vi; ++i) {
      body = index_rows(f.data, f.size, body, f.elems[(size_t)i].count, nullptr, threads);
      if (body == (size_t)-1) return FCCF_E_IO;
    }
    // n rows need n - 1 newlines after the body start: check before the row index is allocated
    if (f.n > 0 && (uint64_t)(f.n - 1) > (uint64_t)(f.size - body)) return FCCF_E_IO;
    if (index_rows(f.data, f.size, body, f.n, &f.rowoff, threads) == (size_t)-1) return FCCF_E_IO;
    return FCCF_OK;
  }
  // binary: walk the elements before the vertex element
  auto walk_row = [&](const Elem& el, size_t& q) -> bool {
    for (const Prop& pr : el.props) {
      if (pr.is_list) {
        if (q + (size_t)pr.csize > f.size) return false;
        const int64_t c = bin_count((const unsigned char*)f.data + q, pr.count_type, swap);
        if (c < 0) return false;
        q += (size_t)pr.csize + (size_t)c * (size_t)pr.size;
      } else {
        q += (size_t)pr.size;
      }
      if (q > f.size) return false;
    }
    return true;
  };
  for (int i = 0; i < f.vi; ++i) {
    const Elem& el = f.elems[(size_t)i];
    if (el.props.empty()) continue;  // zero-byte rows
    for (int64_t r = 0; r < el.count; ++r)
      if (!walk_row(el, body)) return FCCF_E_IO;
  }
  f.vbase = body;
  f.fixed = true;
  int off = 0;
  for (size_t j = 0; j < V.props.size(); ++j) {
    if (V.props[j].is_list) f.fixed = false;
    for (int a = 0; a < 3; ++a)
      if ((int)j == f.xyz[a]) f.off[a] = off;
    off += V.props[j].size;
  }
  f.rec = off;
  // rec <= 8 bytes per property and n < 2^31: the products below cannot wrap in 64 bits
  if (f.fixed) {
    if ((uint64_t)f.rec * (uint64_t)f.n > (uint64_t)(f.size - f.vbase)) return FCCF_E_IO;
    return FCCF_OK;
  }
  // a vertex row holds at least its x, y, z bytes: bound n by the data before allocating
  if ((uint64_t)f.n * 3u > (uint64_t)(f.size - f.vbase)) return FCCF_E_IO;
  f.rowoff.resize((size_t)f.n);
  for (int64_t r = 0; r < f.n; ++r) {
    f.rowoff[(size_t)r] = body;
    if (!walk_row(V, body)) return FCCF_E_IO;
  }
  return FCCF_OK;
}

bool packed_xyz(const File& f) {
  if (f.fmt == File::ASCII || !f.fixed || f.rec != 12 || f.off[0] != 0 || f.off[1] != 4 || f.off[2] != 8) return false;
  const bool swap = (f.fmt == File::LE && !host_little()) || (f.fmt == File::BE && host_little());
  const Elem& V = f.elems[(size_t)f.vi];
  return !swap && is_float(V.props[(size_t)f.xyz[0]].type) && is_float(V.props[(size_t)f.xyz[1]].type) &&
         is_float(V.props[(size_t)f.xyz[2]].type);
}

int decode(const File& f, int64_t r0, int64_t nr, float* out) {
  if (r0 < 0 || nr < 0 || r0 + nr > f.n) return FCCF_E_ARG;
  const Elem& V = f.elems[(size_t)f.vi];
  const unsigned char* d = (const unsigned char*)f.data;
  if (f.fmt != File::ASCII) {
    const bool swap = (f.fmt == File::LE && !host_little()) || (f.fmt == File::BE && host_little());
    const std::string* ty[3] = {&V.props[(size_t)f.xyz[0]].type, &V.props[(size_t)f.xyz[1]].type,
                                &V.props[(size_t)f.xyz[2]].type};
    const bool plain = f.fixed && !swap && f.rec == 12 && f.off[0] == 0 && f.off[1] == 4 && f.off[2] == 8 &&
                       is_float(*ty[0]) && is_float(*ty[1]) && is_float(*ty[2]);
    if (plain) {  // the common layout: packed little-endian float xyz
      std::memcpy(out, d + f.vbase + 12 * (size_t)r0, 12 * (size_t)nr);
      return FCCF_OK;
    }
    for (int64_t r = 0; r < nr; ++r) {
      size_t row;
      int off[3] = {f.off[0], f.off[1], f.off[2]};
      if (f.fixed) {
        row = f.vbase + (size_t)f.rec * (size_t)(r0 + r);
      } else {  // list properties: offsets of x, y, z within this row
        row = f.rowoff[(size_t)(r0 + r)];
        size_t q = 0;
        for (size_t j = 0; j < V.props.size(); ++j) {
          const Prop& pr = V.props[j];
          for (int a = 0; a < 3; ++a)
            if ((int)j == f.xyz[a]) off[a] = (int)q;
          if (pr.is_list) q += (size_t)pr.csize + (size_t)bin_count(d + row + q, pr.count_type, swap) * pr.size;
          else q += (size_t)pr.size;
        }
      }
      for (int a = 0; a < 3; ++a) out[3 * r + a] = bin_value(d + row + off[a], *ty[a], swap);
    }
    return FCCF_OK;
  }
  const char* end = f.data + f.size;
  for (int64_t r = 0; r < nr; ++r) {
    const char* p = f.data + f.rowoff[(size_t)(r0 + r)];
    const char* e = row_end(p, end);
    float v[3] = {0.f, 0.f, 0.f};
    for (size_t j = 0; j < V.props.size(); ++j) {
      const Prop& pr = V.props[j];
      size_t len;
      const char* s = next_token(p, e, len);
      if (pr.is_list) {  // (a row holds at most e - p more tokens)
        const int64_t c = std::min<int64_t>(std::max<int64_t>(count_of(ascii_value(s, len, pr.count_type)), 0), e - p);
        for (int64_t k = 0; k < c; ++k) (void)next_token(p, e, len);
        continue;
      }
      for (int a = 0; a < 3; ++a)
        if ((int)j == f.xyz[a]) v[a] = ascii_value(s, len, pr.type);
    }
    out[3 * r] = v[0];
    out[3 * r + 1] = v[1];
    out[3 * r + 2] = v[2];
  }
  return FCCF_OK;
}

}  // namespace ply
}  // namespace fccf

extern "C" void fccf_free(void* p) { std::free(p); }

extern "C" int fccf_ply_read(const char* path, float** out, int64_t* nout) {
  if (!path || !out || !nout) return FCCF_E_ARG;
  *out = nullptr;
  *nout = 0;
  float* xyz = nullptr;
  // no exception may cross the C ABI (allocation in the header parse or the row index,
  // thread creation): each becomes a status code
  try {
    const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    fccf::ply::File f;
    if (int rc = fccf::ply::open(path, f, T)) return rc;
    xyz = (float*)std::malloc(sizeof(float) * 3 * (size_t)(f.n ? f.n : 1));  // n < 2^31 (open)
    if (!xyz) return FCCF_E_OOM;
    // rows in T contiguous ranges on T threads
    std::vector<int> rc(T, FCCF_OK);
    auto part = [&](int t) {
      const int64_t a = f.n * t / T, b = f.n * (t + 1) / T;
      rc[t] = fccf::ply::decode(f, a, b - a, xyz + 3 * a);
    };
    std::vector<std::thread> th;
    struct Join {  // destroyed before f and rc, also when a thread fails to start
      std::vector<std::thread>& th;
      ~Join() {
        for (auto& x : th)
          if (x.joinable()) x.join();
      }
    } join{th};
    for (int t = 1; t < T; ++t) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
    for (int t = 0; t < T; ++t)
      if (rc[t]) {
        std::free(xyz);
        return rc[t];
      }
    *out = xyz;
    *nout = f.n;
    return FCCF_OK;
  } catch (const std::bad_alloc&) {
    std::free(xyz);
    return FCCF_E_OOM;
  } catch (...) {
    std::free(xyz);
    return FCCF_E_INTERNAL;
  }
}

extern "C" int fccf_ply_write(const char* path, const float* xyz, int64_t n, int binary) {
  if (!path || (!xyz && n) || n < 0) return FCCF_E_ARG;
  FILE* f = std::fopen(path, "wb");
  if (!f) return FCCF_E_IO;
  const uint16_t one = 1;
  const bool little = *(const uint8_t*)&one == 1;
  std::fprintf(f, "ply\nformat %s 1.0\nelement vertex %lld\nproperty float x\nproperty float y\nproperty float z\nend_header\n",
               binary ? (little ? "binary_little_endian" : "binary_big_endian") : "ascii", (long long)n);
  if (binary) {
    std::fwrite(xyz, sizeof(float), 3 * (size_t)n, f);
  } else {
    for (int64_t i = 0; i < n; ++i) std::fprintf(f, "%.9g %.9g %.9g\n", xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
  }
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  return ok ? FCCF_OK : FCCF_E_IO;
}
