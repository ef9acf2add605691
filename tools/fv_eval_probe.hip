// Dev probe: where k_fv_eval's time goes (fine.hip's LDS form of fine_verify).  A copy of
// the kernel with thread 0 stamping s_memrealtime (100 MHz) after each phase, run on
// synthetic entry lists shaped like c3's (E evaluations, ~2600 tile-leaf entries over
// ~1400 distinct leaf codes each).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
// tools/fv_eval_probe.hip -o tools/fv_eval_probe; run: tools/fv_eval_probe [m] [U] [E]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr uint32_t FV_LDS_MAX = 4096, FV_LDS_SLOTS = 2 * FV_LDS_MAX;
constexpr unsigned long long FV_EMPTY = ~0ull;
constexpr int NPH = 8;

__device__ __forceinline__ void stamp(unsigned long long* ph, int k) {
  if (threadIdx.x == 0) ph[blockIdx.x * NPH + k] = __builtin_amdgcn_s_memrealtime();
}


// Bitonic sort of P2 (power of two, <= 4096) packed 64-bit keys held in registers:
// element i lives in thread i % 1024, slot i / 1024.  Partners in the same wave swap by
// shuffles, partners in other waves through LDS (xs, P2 u64), same-thread partners in
// registers.
template <int E>
__device__ __forceinline__ void reg_bitonic(unsigned long long (&v)[E], uint32_t P2, unsigned long long* xs) {
  const uint32_t t = threadIdx.x;
  for (uint32_t k = 2; k <= P2; k <<= 1) {
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      if (jj >= 1024) {
        const uint32_t d = jj >> 10;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const uint32_t rp = (uint32_t)r ^ d;
          if ((uint32_t)r < rp && rp < (uint32_t)E) {
            const uint32_t i = t + 1024u * r;
            const bool asc = (i & k) == 0;
            const unsigned long long a = v[r], b = v[rp];
            const bool sw = asc ? a > b : a < b;
            v[r] = sw ? b : a;
            v[rp] = sw ? a : b;
          }
        }
      } else if (jj >= 64) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const uint32_t i = t + 1024u * r;
          if (i < P2) xs[i] = v[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const uint32_t i = t + 1024u * r;
          if (i < P2) {
            const unsigned long long o = xs[i ^ jj];
            const bool asc = (i & k) == 0, lower = (i & jj) == 0;
            const bool keep_min = asc == lower;
            v[r] = keep_min ? (o < v[r] ? o : v[r]) : (o > v[r] ? o : v[r]);
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const uint32_t i = t + 1024u * r;
          const uint32_t lo = (uint32_t)v[r], hi = (uint32_t)(v[r] >> 32);
          const uint32_t olo = (uint32_t)__shfl_xor((int)lo, (int)jj, 64);
          const uint32_t ohi = (uint32_t)__shfl_xor((int)hi, (int)jj, 64);
          const unsigned long long o = ((unsigned long long)ohi << 32) | olo;
          const bool asc = (i & k) == 0, lower = (i & jj) == 0;
          const bool keep_min = asc == lower;
          v[r] = keep_min ? (o < v[r] ? o : v[r]) : (o > v[r] ? o : v[r]);
        }
      }
    }
  }
}

// similar_num: the sequential float sum of U terms (one lane), groups of 16 without
// per-term conditions, the next group's loads issued before the current adds
__device__ __forceinline__ float seq_sum(const uint32_t* ht, uint32_t U) {
  float s = 0.f;
  const uint4* __restrict__ t4 = reinterpret_cast<const uint4*>(ht);
  const uint32_t full = U & ~15u;
  uint4 cur[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) cur[u] = t4[u];
  for (uint32_t g = 0; g < full; g += 16) {
    uint4 nxt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) nxt[u] = t4[((g + 16) >> 2) + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s += __uint_as_float(cur[u].x);
      s += __uint_as_float(cur[u].y);
      s += __uint_as_float(cur[u].z);
      s += __uint_as_float(cur[u].w);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
  }
  for (uint32_t g = full; g < U; ++g) s += __uint_as_float(ht[g]);
  return s;
}

// mode bit 0: skip the bitonic network (timing only); bit 1: one wave sums (no other change)
__global__ void __launch_bounds__(1024) k_eval(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                               uint32_t m, uint32_t n, float* __restrict__ scores,
                                               unsigned long long* __restrict__ ph, int mode) {
  __shared__ unsigned long long hk[FV_LDS_SLOTS];
  __shared__ uint32_t hs[FV_LDS_SLOTS];
  __shared__ __attribute__((aligned(16))) uint32_t ht[FV_LDS_SLOTS];
  __shared__ uint32_t snu, sover;
  const int e = blockIdx.x;
  stamp(ph, 0);
  const uint64_t* __restrict__ ke = keys + (size_t)e * n;
  const uint32_t* __restrict__ ve = vals + (size_t)e * n;
  for (uint32_t j = threadIdx.x; j < FV_LDS_SLOTS; j += 1024) {
    hk[j] = FV_EMPTY;
    hs[j] = 0u;
    ht[j] = 0u;
  }
  if (threadIdx.x == 0) {
    snu = 0u;
    sover = 0u;
  }
  __syncthreads();
  stamp(ph, 1);
  for (uint32_t j = threadIdx.x; j < m; j += 1024) {
    const unsigned long long key = ke[j];
    const uint32_t c = ve[j];
    uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 51);
    bool ok = false;
    for (uint32_t probe = 0; probe < FV_LDS_SLOTS; ++probe) {
      const unsigned long long old = atomicCAS(&hk[h], FV_EMPTY, key);
      if (old == FV_EMPTY) {
        if (atomicAdd(&snu, 1u) >= FV_LDS_MAX) sover = 1u;
        ok = true;
        break;
      }
      if (old == key) {
        ok = true;
        break;
      }
      h = (h + 1u) & (FV_LDS_SLOTS - 1u);
    }
    if (!ok) {
      sover = 1u;
      continue;
    }
    atomicAdd(&hs[h], c & 0xFFFFu);
    atomicAdd(&ht[h], c >> 16);
  }
  __syncthreads();
  stamp(ph, 2);
  const uint32_t U = snu;
  {
    constexpr uint32_t PER = FV_LDS_SLOTS / 1024;
    unsigned long long k8[PER];
    uint32_t s8[PER], t8[PER], occ = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t j = threadIdx.x * PER + q;
      k8[q] = hk[j];
      s8[q] = hs[j];
      t8[q] = ht[j];
      occ += k8[q] != FV_EMPTY ? 1u : 0u;
    }
    __shared__ uint32_t wsum[16];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x = occ;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t pos = x - occ;
    for (uint32_t w = 0; w < wave; ++w) pos += wsum[w];
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q)
      if (k8[q] != FV_EMPTY) {
        hk[pos] = k8[q];
        hs[pos] = s8[q];
        ht[pos] = t8[q];
        ++pos;
      }
  }
  __syncthreads();
  stamp(ph, 3);
  uint32_t P2 = 2;
  while (P2 < U) P2 <<= 1;
  for (uint32_t i = threadIdx.x; i < P2; i += 1024) {
    if (i < U) {
      const float sn = (float)hs[i], tn = (float)ht[i];
      float t = 0.f;
      if (sn >= 1.f && tn >= 1.f) {
        const float mn = sn < tn ? sn : tn, mx = sn > tn ? sn : tn;
        t = (sn + tn) * (mn / mx);
      }
      ht[i] = __float_as_uint(t);
    } else {
      hk[i] = FV_EMPTY;
    }
  }
  __syncthreads();
  stamp(ph, 4);
  if (mode == 2) {  // packed (code << 32 | term) keys sorted in registers, then the sum
    unsigned long long v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t i = threadIdx.x + 1024u * r;
      v[r] = i < U ? (hk[i] << 32) | ht[i] : ~0ull;
    }
    __syncthreads();
    unsigned long long* xs = hk;  // (the codes are in registers now)
    if (P2 <= 1024) {
      unsigned long long a[1] = {v[0]};
      reg_bitonic<1>(a, P2, xs);
      v[0] = a[0];
    } else if (P2 <= 2048) {
      unsigned long long a[2] = {v[0], v[1]};
      reg_bitonic<2>(a, P2, xs);
      v[0] = a[0];
      v[1] = a[1];
    } else {
      reg_bitonic<4>(v, P2, xs);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t i = threadIdx.x + 1024u * r;
      if (i < U) ht[i] = (uint32_t)v[r];
    }
    __syncthreads();
    stamp(ph, 5);
    if (threadIdx.x == 0) {
      scores[e] = seq_sum(ht, U);
      ph[blockIdx.x * NPH + 6] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  if (!(mode & 1))
    for (uint32_t k = 2; k <= P2; k <<= 1) {
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        if (jj >= 128) {
          __syncthreads();
        } else {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (uint32_t c = threadIdx.x; c < P2 / 2; c += 1024) {
          const uint32_t i = ((c & ~(jj - 1)) << 1) | (c & (jj - 1)), l = i | jj;
          const unsigned long long a = hk[i], b = hk[l];
          if (((i & k) == 0) ? a > b : a < b) {
            hk[i] = b;
            hk[l] = a;
            const uint32_t t0 = ht[i];
            ht[i] = ht[l];
            ht[l] = t0;
          }
        }
        if (jj >= 128) __syncthreads();
      }
    }
  __syncthreads();
  stamp(ph, 5);
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  if (lane == 0) {
    float similar = 0.f;
    const uint4* __restrict__ t4 = reinterpret_cast<const uint4*>(ht);
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = t4[u];
    for (uint32_t g = 0; g < U; g += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) nxt[u] = t4[((g + 16) >> 2) + u];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (g + 4 * u + 0 < U) similar += __uint_as_float(cur[u].x);
        if (g + 4 * u + 1 < U) similar += __uint_as_float(cur[u].y);
        if (g + 4 * u + 2 < U) similar += __uint_as_float(cur[u].z);
        if (g + 4 * u + 3 < U) similar += __uint_as_float(cur[u].w);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
    }
    scores[e] = similar;
    ph[blockIdx.x * NPH + 6] = __builtin_amdgcn_s_memrealtime();
  }
}

int main(int argc, char** argv) {
  const uint32_t m = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 2624u;
  const uint32_t U = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1400u;
  const int E = argc > 3 ? std::atoi(argv[3]) : 12;
  const uint32_t n = m + 64;
  std::mt19937_64 rng(5);
  std::vector<uint64_t> keys((size_t)E * n, 0);
  std::vector<uint32_t> vals((size_t)E * n, 0);
  for (int e = 0; e < E; ++e) {
    std::vector<uint64_t> codes(U);
    for (auto& c : codes) c = rng() & ((1ull << 27) - 1);  // 9-level morton codes
    for (uint32_t j = 0; j < m; ++j) {
      keys[(size_t)e * n + j] = codes[j < U ? j : rng() % U];
      vals[(size_t)e * n + j] = (uint32_t)(rng() % 40) | ((uint32_t)(rng() % 40) << 16);
    }
    std::shuffle(keys.begin() + (size_t)e * n, keys.begin() + (size_t)e * n + m, rng);
  }
  uint64_t* dk;
  uint32_t* dv;
  float* ds;
  unsigned long long* dph;
  CK(hipMalloc(&dk, 8 * keys.size()));
  CK(hipMalloc(&dv, 4 * vals.size()));
  CK(hipMalloc(&ds, 4 * E));
  CK(hipMalloc(&dph, 8 * NPH * E));
  CK(hipMemcpy(dk, keys.data(), 8 * keys.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, vals.data(), 4 * vals.size(), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[] = {"init", "merge", "compact", "terms", "bitonic", "sum"};
  std::vector<float> sc0(E), sc2(E);
  for (int mode : {0, 1, 2}) {
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemset(dph, 0, 8 * NPH * E));
      CK(hipEventRecord(a, 0));
      k_eval<<<E, 1024>>>(dk, dv, m, n, ds, dph, mode);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      std::vector<unsigned long long> ph(NPH * E);
      CK(hipMemcpy(ph.data(), dph, 8 * ph.size(), hipMemcpyDeviceToHost));
      if (rep < 3) continue;
      if (mode == 0) CK(hipMemcpy(sc0.data(), ds, 4 * E, hipMemcpyDeviceToHost));
      if (mode == 2) {
        CK(hipMemcpy(sc2.data(), ds, 4 * E, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int q = 0; q < E; ++q) bad += std::memcmp(&sc0[q], &sc2[q], 4) != 0;
        std::printf("mode 2 scores vs mode 0: %d of %d differ\n", bad, E);
      }
      std::printf("mode %d (m %u, U %u, E %d): kernel %.1f us (events); per phase, us (workgroup 0 / max):", mode, m, U,
                  E, ms * 1e3);
      for (int k = 0; k < 6; ++k) {
        double mx = 0;
        for (int e = 0; e < E; ++e) mx = std::max(mx, (double)(ph[e * NPH + k + 1] - ph[e * NPH + k]) * 1e-2);
        std::printf(" %s %.2f/%.2f", names[k], (double)(ph[k + 1] - ph[k]) * 1e-2, mx);
      }
      std::printf("\n");
    }
  }
  return 0;
}
