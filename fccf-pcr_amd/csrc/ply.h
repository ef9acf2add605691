// ply.h — PLY vertex decoding shared by fccf_ply_read (host arrays) and the
// streaming ingest (ingest.cpp).  Reference surface:
// pcl::io::loadPLYFile<PointXYZ> in main (FCCF.cpp:1655-1665): the vertex element's
// x, y, z by name, in file order; every other property and element is skipped.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fccf {
namespace ply {

struct Prop {
  std::string name, type, count_type;
  bool is_list = false;
  int size = 0, csize = 0;  // bytes of the value type / the list count type
};
struct Elem {
  std::string name;
  int64_t count = 0;
  std::vector<Prop> props;
};

// A mapped PLY file and the layout of its vertex rows.
struct File {
  int fd = -1;
  const char* data = nullptr;
  size_t size = 0;
  enum Fmt { ASCII, LE, BE } fmt = ASCII;
  std::vector<Elem> elems;
  int vi = -1;          // index of the vertex element
  int64_t n = 0;        // vertex count
  int xyz[3] = {-1, -1, -1};  // property index of x, y, z in the vertex element
  // binary: vertex rows start at vbase; fixed-size rows (no list property) have
  // stride rec and x/y/z at byte offsets off[]; otherwise rows are walked (rowoff)
  size_t vbase = 0;
  int rec = 0, off[3] = {0, 0, 0};
  bool fixed = false;
  // ascii, and binary rows of variable size: byte offset of every vertex row
  std::vector<size_t> rowoff;
  ~File();
};

// Maps path and parses the header (and, where rows are not fixed-size, indexes the
// vertex rows, with `threads` threads).  FCCF_OK or FCCF_E_IO / FCCF_E_OOM.
int open(const char* path, File& f, int threads);
// Rows [r0, r0 + nr) as float xyz into out (3 * nr floats).  FCCF_OK or FCCF_E_IO
// (a malformed ascii row).  Safe to call concurrently on disjoint ranges.
int decode(const File& f, int64_t r0, int64_t nr, float* out);
// The vertex rows are packed host-endian float x, y, z (12 B rows): the mapped bytes
// from f.vbase are the decoded cloud.
bool packed_xyz(const File& f);

}  // namespace ply
}  // namespace fccf
