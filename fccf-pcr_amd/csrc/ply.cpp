// ply.cpp — PLY reader/writer for the CLI surface of FCCF.cpp:1655-1665
// (pcl::io::loadPLYFile<PointXYZ>): ascii, binary_little_endian and
// binary_big_endian vertex elements; x, y, z mapped by name (float32, or float64
// narrowed); every other property (and every other element) is skipped by size.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/fccf.h"

namespace {

struct Prop {
  std::string name, type;
  bool is_list = false;
  std::string count_type;
};
struct Elem {
  std::string name;
  int64_t count = 0;
  std::vector<Prop> props;
};

int type_size(const std::string& t) {
  if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
  if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
  if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
  if (t == "double" || t == "float64") return 8;
  return 0;
}

double read_bin(const unsigned char* p, const std::string& t, bool swap) {
  unsigned char b[8];
  const int s = type_size(t);
  for (int i = 0; i < s; ++i) b[i] = swap ? p[s - 1 - i] : p[i];
  if (t == "char" || t == "int8") return (double)*(int8_t*)b;
  if (t == "uchar" || t == "uint8") return (double)*(uint8_t*)b;
  if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); return v; }
  if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); return v; }
  if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); return v; }
  if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); return v; }
  if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); return v; }
  double v;
  std::memcpy(&v, b, 8);
  return v;
}

bool host_little() {
  const uint16_t x = 1;
  return *(const uint8_t*)&x == 1;
}

}  // namespace

extern "C" void fccf_free(void* p) { std::free(p); }

extern "C" int fccf_ply_read(const char* path, float** out, int64_t* nout) {
  if (!path || !out || !nout) return FCCF_E_ARG;
  *out = nullptr;
  *nout = 0;
  std::ifstream f(path, std::ios::binary);
  if (!f) return FCCF_E_IO;
  std::string line;
  if (!std::getline(f, line) || line.compare(0, 3, "ply") != 0) return FCCF_E_IO;
  std::string format;
  std::vector<Elem> elems;
  while (std::getline(f, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::istringstream ss(line);
    std::string kw;
    ss >> kw;
    if (kw == "format") ss >> format;
    else if (kw == "element") {
      Elem e;
      ss >> e.name >> e.count;
      elems.push_back(e);
    } else if (kw == "property") {
      if (elems.empty()) return FCCF_E_IO;
      Prop p;
      std::string t;
      ss >> t;
      if (t == "list") {
        p.is_list = true;
        ss >> p.count_type >> p.type >> p.name;
      } else {
        p.type = t;
        ss >> p.name;
      }
      elems.back().props.push_back(p);
    } else if (kw == "end_header") {
      break;
    }
  }
  const bool ascii = format == "ascii";
  const bool le = format == "binary_little_endian", be = format == "binary_big_endian";
  if (!ascii && !le && !be) return FCCF_E_IO;
  const bool swap = (le && !host_little()) || (be && host_little());
  int64_t nv = 0;
  for (auto& e : elems)
    if (e.name == "vertex") nv = e.count;
  float* xyz = (float*)std::malloc(sizeof(float) * 3 * (size_t)(nv ? nv : 1));
  if (!xyz) return FCCF_E_OOM;
  bool have[3] = {false, false, false};
  for (auto& e : elems) {
    if (e.name != "vertex") continue;
    for (auto& p : e.props) {
      if (p.name == "x") have[0] = true;
      if (p.name == "y") have[1] = true;
      if (p.name == "z") have[2] = true;
    }
  }
  if (!(have[0] && have[1] && have[2])) { std::free(xyz); return FCCF_E_IO; }
  for (auto& e : elems) {
    const bool isv = e.name == "vertex";
    for (int64_t r = 0; r < e.count; ++r) {
      if (ascii) {
        if (!std::getline(f, line)) { std::free(xyz); return FCCF_E_IO; }
        std::istringstream ss(line);
        for (auto& p : e.props) {
          if (p.is_list) {
            double c; ss >> c;
            for (int64_t k = 0; k < (int64_t)c; ++k) { double d; ss >> d; }
            continue;
          }
          double v;
          if (!(ss >> v)) { std::free(xyz); return FCCF_E_IO; }
          if (isv) {
            if (p.name == "x") xyz[3 * r] = (float)v;
            else if (p.name == "y") xyz[3 * r + 1] = (float)v;
            else if (p.name == "z") xyz[3 * r + 2] = (float)v;
          }
        }
      } else {
        unsigned char buf[8];
        for (auto& p : e.props) {
          if (p.is_list) {
            const int cs = type_size(p.count_type), es = type_size(p.type);
            if (!cs || !es || !f.read((char*)buf, cs)) { std::free(xyz); return FCCF_E_IO; }
            const int64_t c = (int64_t)read_bin(buf, p.count_type, swap);
            f.seekg(c * es, std::ios::cur);
            continue;
          }
          const int s = type_size(p.type);
          if (!s || !f.read((char*)buf, s)) { std::free(xyz); return FCCF_E_IO; }
          if (isv) {
            const double v = read_bin(buf, p.type, swap);
            if (p.name == "x") xyz[3 * r] = (float)v;
            else if (p.name == "y") xyz[3 * r + 1] = (float)v;
            else if (p.name == "z") xyz[3 * r + 2] = (float)v;
          }
        }
      }
    }
  }
  *out = xyz;
  *nout = nv;
  return FCCF_OK;
}

extern "C" int fccf_ply_write(const char* path, const float* xyz, int64_t n, int binary) {
  if (!path || (!xyz && n) || n < 0) return FCCF_E_ARG;
  FILE* f = std::fopen(path, "wb");
  if (!f) return FCCF_E_IO;
  std::fprintf(f, "ply\nformat %s 1.0\nelement vertex %lld\nproperty float x\nproperty float y\nproperty float z\nend_header\n",
               binary ? (host_little() ? "binary_little_endian" : "binary_big_endian") : "ascii", (long long)n);
  if (binary) {
    std::fwrite(xyz, sizeof(float), 3 * (size_t)n, f);
  } else {
    for (int64_t i = 0; i < n; ++i) std::fprintf(f, "%.9g %.9g %.9g\n", xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
  }
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  return ok ? FCCF_OK : FCCF_E_IO;
}
