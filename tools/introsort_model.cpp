// introsort_model.cpp — development model (not product, not oracle) of the GPU
// reproduction of libstdc++ std::sort (introsort) on PCL VoxelGrid's
// (idx, cloud_point_index) pairs compared by idx only (FCCF.cpp:1668-1678 via
// pcl::VoxelGrid::applyFilter).
//
// Checks, against std::sort of this toolchain, that the partition of a segment can
// be computed from prefix counts alone (no sequential scan):
//   after __move_median_to_first(first, first+1, mid, last-1) with pivot P at first,
//   __unguarded_partition(first+1, last, first) swaps the k-th element >= P from the
//   left (L[k]) with the k-th element <= P from the right (R[k]) for every k with
//   L[k] < R[k] (a prefix k = 1..K), and returns cut = min(L[K+1], R[K]) (R[0] = last).
// An element >= P at position p with ge-rank k is swapped iff #(<=P after p) >= k;
// an element <= P with right-rank k is swapped iff #(>=P before it) >= k.
// The final insertion sort is stable, and every leaf segment (<= 16 elements, or
// heap-sorted at depth 0) is bounded by its neighbours, so the result is the
// concatenation of the stable sorts of the leaf segments.
//
// Build: g++ -O2 -std=c++17 tools/introsort_model.cpp -o /tmp/introsort_model
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

struct E {
  uint32_t key, val;
  bool operator<(const E& o) const { return key < o.key; }
};

static int lg(size_t n) { return 63 - __builtin_clzll(n); }

// heap sort exactly as std::__partial_sort(first, last, last) (make_heap, sort_heap)
static void adjust_heap(E* a, long hole, long len, E v) {
  const long top = hole;
  long sc = hole;
  while (sc < (len - 1) / 2) {
    sc = 2 * (sc + 1);
    if (a[sc].key < a[sc - 1].key) sc--;
    a[hole] = a[sc];
    hole = sc;
  }
  if ((len & 1) == 0 && sc == (len - 2) / 2) {
    sc = 2 * (sc + 1);
    a[hole] = a[sc - 1];
    hole = sc - 1;
  }
  long parent = (hole - 1) / 2;
  while (hole > top && a[parent].key < v.key) {
    a[hole] = a[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a[hole] = v;
}
static void heap_sort(E* a, long len) {
  if (len < 2) return;
  for (long parent = (len - 2) / 2;; parent--) {
    adjust_heap(a, parent, len, a[parent]);
    if (parent == 0) break;
  }
  for (long last = len - 1; last > 0; --last) {
    E v = a[last];
    a[last] = a[0];
    adjust_heap(a, 0, last, v);
  }
}

struct Seg {
  size_t f, l;
  int depth;
};

// one partition of [f,l) by the prefix-count rule; returns the cut
static size_t partition_counts(std::vector<E>& a, size_t f, size_t l) {
  const size_t mid = f + (l - f) / 2;
  const size_t A = f + 1, B = mid, C = l - 1;
  size_t m;  // __move_median_to_first(f, A, B, C)
  if (a[A].key < a[B].key) {
    if (a[B].key < a[C].key) m = B;
    else if (a[A].key < a[C].key) m = C;
    else m = A;
  } else if (a[A].key < a[C].key) m = A;
  else if (a[B].key < a[C].key) m = C;
  else m = B;
  std::swap(a[f], a[m]);
  const uint32_t P = a[f].key;
  const size_t n = l - (f + 1);
  std::vector<uint32_t> gepre(n + 1, 0), lepre(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    gepre[i + 1] = gepre[i] + (a[f + 1 + i].key >= P);
    lepre[i + 1] = lepre[i] + (a[f + 1 + i].key <= P);
  }
  const uint32_t letot = lepre[n];
  std::vector<size_t> Lk(n + 2, l), Rk(n + 2, l);  // L[k], R[k] positions (1-based k)
  std::vector<E> out(a.begin() + f, a.begin() + l);
  size_t cut = l;
  for (size_t i = 0; i < n; ++i) {
    const size_t p = f + 1 + i;
    const uint32_t key = a[p].key;
    if (key >= P) {
      const uint32_t k = gepre[i + 1];
      const uint32_t le_after = letot - lepre[i + 1];
      if (le_after >= k) Lk[k] = p;
      else cut = std::min(cut, p);  // first non-swapped >= element = L[K+1]
    }
    if (key <= P) {
      const uint32_t k = letot - lepre[i];  // right rank
      const uint32_t ge_before = gepre[i];
      if (ge_before >= k) {
        Rk[k] = p;
        cut = std::min(cut, p);  // R[K] = the smallest swapped <= position
      }
    }
  }
  for (size_t k = 1; k <= n && Lk[k] != l; ++k) {
    if (Rk[k] == l) { std::fprintf(stderr, "unpaired swap\n"); std::abort(); }
    out[Rk[k] - f] = a[Lk[k]];
    out[Lk[k] - f] = a[Rk[k]];
  }
  std::copy(out.begin(), out.end(), a.begin() + f);
  return cut;
}

// the round-based model: every segment > 16 of a round is partitioned; returns rounds
static int model_sort(std::vector<E>& a, size_t tier, int* rounds_to_tier) {
  if (a.empty()) return 0;
  std::vector<Seg> cur{{0, a.size(), 2 * lg(a.size())}}, leaves;
  int rounds = 0;
  *rounds_to_tier = -1;
  while (!cur.empty()) {
    size_t mx = 0;
    for (auto& s : cur) mx = std::max(mx, s.l - s.f);
    if (*rounds_to_tier < 0 && mx <= tier) *rounds_to_tier = rounds;
    if (std::getenv("MODEL_TRACE") && *rounds_to_tier < 0) {
      size_t nl = 0, tot = 0;
      for (auto& s : cur) if (s.l - s.f > tier) { ++nl; tot += s.l - s.f; }
      std::printf("  round %d: %zu segments > %zu, %zu elements, max %zu\n", rounds, nl, tier, tot, mx);
    }
    std::vector<Seg> nxt;
    for (auto& s : cur) {
      if (s.l - s.f <= 16) { leaves.push_back(s); continue; }
      if (s.depth == 0) {
        heap_sort(a.data() + s.f, (long)(s.l - s.f));
        leaves.push_back(s);
        continue;
      }
      const size_t c = partition_counts(a, s.f, s.l);
      nxt.push_back({c, s.l, s.depth - 1});
      nxt.push_back({s.f, c, s.depth - 1});
    }
    cur.swap(nxt);
    ++rounds;
  }
  for (auto& s : leaves) std::stable_sort(a.begin() + s.f, a.begin() + s.l);
  return rounds;
}

// McIlroy's adversary: a comparison-consistent input that drives std::sort deep
static std::vector<uint32_t> killer(size_t n) {
  std::vector<int> val(n, -1);
  std::vector<uint32_t> idx(n);
  for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
  int gas = (int)n, nsolid = 0, candidate = 0;
  auto freeze = [&](int x) { val[x] = nsolid++; };
  std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) {
    if (val[x] < 0 && val[y] < 0) { if ((int)x == candidate) freeze(x); else freeze(y); }
    if (val[x] < 0) candidate = x;
    else if (val[y] < 0) candidate = y;
    int vx = val[x] < 0 ? gas : val[x], vy = val[y] < 0 ? gas : val[y];
    return vx < vy;
  });
  std::vector<uint32_t> keys(n);
  for (size_t i = 0; i < n; ++i) keys[i] = (uint32_t)(val[i] < 0 ? gas : val[i]);
  return keys;
}

static bool check(const std::vector<uint32_t>& keys, size_t tier, int* rounds, int* rt) {
  std::vector<E> a(keys.size()), b;
  for (size_t i = 0; i < keys.size(); ++i) a[i] = {keys[i], (uint32_t)i};
  b = a;
  std::sort(a.begin(), a.end());
  *rounds = model_sort(b, tier, rt);
  return std::memcmp(a.data(), b.data(), a.size() * sizeof(E)) == 0;
}

int main(int argc, char** argv) {
  std::mt19937_64 rng(12345);
  int bad = 0, tests = 0, r, rt;
  for (int t = 0; t < 3000; ++t) {
    const size_t n = (t < 200) ? (size_t)t : (size_t)(rng() % 5000);
    const uint32_t range = 1 + (uint32_t)(rng() % (t % 3 == 0 ? 4 : (t % 3 == 1 ? 64 : 1u << 30)));
    std::vector<uint32_t> k(n);
    for (auto& x : k) x = (uint32_t)(rng() % range);
    if (t % 7 == 0) std::sort(k.begin(), k.end());
    if (t % 11 == 0) std::sort(k.rbegin(), k.rend());
    ++tests;
    if (!check(k, 8192, &r, &rt)) { ++bad; std::printf("mismatch n=%zu range=%u\n", n, range); }
  }
  for (size_t n : {64, 100, 1000, 4096, 20000}) {
    ++tests;
    if (!check(killer(n), 8192, &r, &rt)) { ++bad; std::printf("killer mismatch n=%zu\n", n); }
    else std::printf("killer n=%zu ok, rounds %d\n", n, r);
  }
  std::printf("%d/%d equal to std::sort\n", tests - bad, tests);
  // rounds statistics on large random-ish leaf keys
  if (argc > 1) {
    FILE* fp = std::fopen(argv[1], "rb");
    if (fp) {
      std::vector<uint32_t> k;
      uint32_t x;
      while (std::fread(&x, 4, 1, fp) == 1) k.push_back(x);
      std::fclose(fp);
      for (size_t tier : {4096, 8192, 16384}) {
        bool ok = check(k, tier, &r, &rt);
        std::printf("file n=%zu tier %zu: equal %d, rounds total %d, rounds to tier %d\n", k.size(), tier, ok, r, rt);
      }
    }
  }
  return bad != 0;
}
