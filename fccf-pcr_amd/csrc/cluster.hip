// cluster.hip — f3: transform_cluster's seed pass, range_cluster's
// exchange sort and the cluster averaging on the GPU (FCCF.cpp:1040-1231, :1020-1038,
// average_normal :325-367), bit-identical to the host form (host_stages.cpp
// transform_cluster, device-rows branch).  Input: k_cluster_bits's neighbour rows.
//
// k_cluster_seeds (one wave per candidate type):
//   * seed pass: the next unallocated candidate (ballot over the allocation words)
//     seeds a cluster; its row is OR-ed into the allocation words and popcounted
//     (the last candidate never seeds, :1084);
//   * range_cluster: the reference's exchange sort (for a, for b > a: swap when
//     x[a] < x[b]) of the clusters of size >= min(max, 2), emulated one outer step at
//     a time by the wave: the swaps of step a happen exactly at the strict prefix
//     maxima of x[a..], and they rotate the record holders one record to the right,
//     so a max-with-argmax scan over x[a+1..] applies the whole step; steps run only
//     as far as the emission loop reads;
//   * the emission loop (:1205-1229): which clusters are averaged, in order.
// k_cluster_avg (one wave per emitted cluster): members = the seed's row, sorted by
//   (d2, j) as the radius search returns them; their sums in that order (one lane,
//   from LDS); normalize, axes_to_rot, quaternion (fccf_math.h).
#define KT_TU 12  // ktrace.h source tag
#include "ktrace.h"
#include "kernels.h"
#include "match.h"

namespace fccf {
namespace {

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

constexpr uint32_t CL_WMAX = 1024;   // allocation words per type (65536 candidates = MatchMail::Q_CAP)
constexpr uint32_t CL_RMAX = 10240;  // row words cached in LDS (80 KB): the seed pass's serial reads

struct TypeRows {
  uint32_t n, W;
  uint64_t off;  // word offset of the type's rows (k_cluster_bits layout)
  bool present;
};
__device__ __forceinline__ TypeRows type_rows(const ClusterIn& in, int t) {
  uint64_t words = 0, off = 0;
  for (int u = 0; u < 3; ++u) {
    const uint64_t n = in.totals[u], w = ((n + 63) / 64) * n;
    if (u < t) off += w;
    words += w;
  }
  TypeRows r;
  r.n = in.totals[t];
  r.W = (r.n + 63) / 64;
  r.off = off;
  r.present = words <= in.cb_cap;
  return r;
}

__global__ void __launch_bounds__(64) k_cluster_seeds(ClusterIn in, ClusterOut out) {
  KT();
  __shared__ uint64_t A[CL_WMAX];
  __shared__ uint64_t R[CL_RMAX];
  const int t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TypeRows ti = type_rows(in, t);
  const uint32_t n = ti.n, W = ti.W;
  // cluster_num as the caller computes it (:1458): int(sel * n / int(total))
  const int tn = (int)(in.totals[0] + in.totals[1] + in.totals[2]);
  const int cnum = in.has_cnum ? in.cnum_given : (tn ? (int)(in.sel * (float)n / (float)tn) : 0);
  const bool mine = ti.present && !((float)n <= in.min_n) && W <= CL_WMAX && n <= out.cap &&
                    (int64_t)cnum + 1 <= (int64_t)out.egrid;
  uint32_t* stat = out.stat + 4 * t;
  if (lane == 0) {
    stat[0] = mine ? 0u : 1u;
    stat[1] = 0;
    stat[2] = 0;
    stat[3] = (uint32_t)cnum;
  }
  if (!mine || n == 0) return;
  const uint64_t* rows = in.rows + ti.off;
  if ((uint64_t)n * W <= CL_RMAX) {  // small sets: the rows into LDS, read serially from there
    for (uint32_t k = lane; k < n * W; k += 64) R[k] = rows[k];
    rows = R;
  }
  uint32_t* cseed = out.cseed[t];
  uint32_t* csize = out.csize[t];
  for (uint32_t w = lane; w < W; w += 64) A[w] = 0ull;
  wsync();
  // ---- seed pass
  uint32_t ncl = 0, mx = 0, cur = 0;
  while (cur + 1 < n) {
    // first candidate >= cur not yet allocated
    uint32_t found = 0xFFFFFFFFu;
    for (uint32_t w0 = cur >> 6; w0 < W && found == 0xFFFFFFFFu; w0 += 64) {
      const uint32_t w = w0 + lane;
      uint64_t free_bits = 0;
      if (w < W) {
        free_bits = ~A[w];
        if (w == (cur >> 6)) free_bits &= ~0ull << (cur & 63);
      }
      const uint64_t bw = __ballot(free_bits != 0);
      if (bw) {
        const uint32_t l0 = (uint32_t)__builtin_ctzll(bw);
        const uint64_t fb = __shfl(free_bits, (int)l0, 64);
        found = (w0 + l0) * 64 + (uint32_t)__builtin_ctzll(fb);
      }
    }
    if (found == 0xFFFFFFFFu || found + 1 >= n) break;  // the last candidate never seeds
    const uint64_t* row = rows + (size_t)found * W;
    uint32_t c = 0;
    for (uint32_t w = lane; w < W; w += 64) {
      const uint64_t rw = row[w];
      A[w] |= rw;
      c += (uint32_t)__popcll(rw);
    }
    c = wave_sum(c);
    if (lane == 0) {
      cseed[ncl] = found;
      csize[ncl] = c;
    }
    mx = max(mx, c);
    ++ncl;
    cur = found + 1;
    wsync();
  }
  if (lane == 0) stat[1] = ncl;
  if (ncl == 0) return;
  // ---- range_cluster: the clusters of size >= thr in creation order (x = size, id = index)
  const uint32_t thr = min(mx, 2u);
  uint32_t* bx = out.bx[t];
  uint32_t* bid = out.bid[t];
  uint32_t B = 0;
  for (uint32_t k0 = 0; k0 < ncl; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool big = k < ncl && csize[k] >= thr;
    const uint64_t bb = __ballot(big);
    if (big) {
      const uint32_t pos = B + (uint32_t)__popcll(bb & ((1ull << lane) - 1ull));
      bx[pos] = csize[k];
      bid[pos] = k;
    }
    B += (uint32_t)__popcll(bb);
  }
  // the rest (sizes < thr <= 2) sorted descending: their ones, then their zeros (a
  // candidate whose x axis is not within the angle of itself has an empty row)
  uint32_t nones = 0;
  for (uint32_t k0 = 0; k0 < ncl; k0 += 64) {
    const uint32_t k = k0 + lane;
    nones += (uint32_t)__popcll(__ballot(k < ncl && csize[k] < thr && csize[k] == 1u));
  }
  wsync();
  // ---- emission loop, with the exchange sort's outer steps applied as needed
  uint32_t clusternum = mx, nemit = 0, sorted = 0;
  for (uint32_t r = 0; r < ncl; ++r) {
    uint32_t size_r;
    if (r < B) {
      while (sorted <= r) {  // outer step a = sorted: x[a] <- max of x[a..]; records rotate right
        const uint32_t a = sorted;
        uint32_t cv = bx[a], ci = bid[a];  // running (max, holder) before each chunk
        for (uint32_t b0 = a + 1; b0 < B; b0 += 64) {
          const uint32_t b = b0 + lane;
          const uint32_t xv = b < B ? bx[b] : 0u, xi = b < B ? bid[b] : 0u;
          // inclusive (max, first holder) over this chunk, strictly-greater replaces
          uint32_t mv = xv, mi = xi;
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t pv = (uint32_t)__shfl_up((int)mv, o, 64), pi = (uint32_t)__shfl_up((int)mi, o, 64);
            if (lane >= (uint32_t)o && !(mv > pv)) {
              mv = pv;
              mi = pi;
            }
          }
          // exclusive prefix with the carry: the max before b and its (first) holder
          uint32_t ev = (uint32_t)__shfl_up((int)mv, 1, 64), ei = (uint32_t)__shfl_up((int)mi, 1, 64);
          if (lane == 0 || !(ev > cv)) {
            ev = cv;
            ei = ci;
          }
          const bool rec = b < B && xv > ev;  // a strict new maximum: the reference swaps here
          wsync();
          if (rec) {
            bx[b] = ev;
            bid[b] = ei;
          }
          // carry: the chunk's overall max (the last lane's inclusive value vs the carry)
          const uint32_t lv = (uint32_t)__shfl((int)mv, 63, 64), li = (uint32_t)__shfl((int)mi, 63, 64);
          if (lv > cv) {
            cv = lv;
            ci = li;
          }
          wsync();
        }
        if (lane == 0) {
          bx[a] = cv;
          bid[a] = ci;
        }
        wsync();
        ++sorted;
      }
      size_r = bx[r];
    } else {
      size_r = r - B < nones ? 1u : 0u;  // rest_sizes[r - B]
    }
    if (size_r >= clusternum) {  // (then r < B: clusternum >= thr)
      if (lane == 0) out.emit[t][nemit] = bid[r];
      ++nemit;
      if ((int64_t)nemit > (int64_t)cnum) break;
    } else {
      if ((double)nemit < ((double)cnum / 2.0)) {
        clusternum--;
        if (clusternum < 2) break;
      } else {
        break;
      }
    }
  }
  if (lane == 0) stat[2] = nemit;
}

constexpr uint32_t CL_MMAX = 1024;  // members held in LDS per emitted cluster

// One wave per emitted cluster (blockIdx.x = emission index, blockIdx.y = type).
__global__ void __launch_bounds__(64) k_cluster_avg(ClusterIn in, ClusterOut out) {
  KT();
  __shared__ uint64_t key[CL_MMAX];  // (d2 bits, j): d2 >= 0, so its bits order as unsigned
  __shared__ float mtx[CL_MMAX], mty[CL_MMAX], mtz[CL_MMAX];
  __shared__ float mq[CL_MMAX][4];
  const int t = blockIdx.y;
  const uint32_t e = blockIdx.x, lane = threadIdx.x;
  uint32_t* stat = out.stat + 4 * t;
  if (stat[0] || e >= stat[2]) return;
  const TypeRows ti = type_rows(in, t);
  const uint32_t W = ti.W;
  const uint32_t k = out.emit[t][e];
  const uint32_t i = out.cseed[t][k];
  const uint64_t* row = in.rows + ti.off + (size_t)i * W;
  const QTd* q = in.q[t];
  const QTd qi = q[i];
  // members in j order, compacted by ballot
  uint32_t cnt = 0;
  for (uint32_t w0 = 0; w0 < W; w0 += 64) {
    const uint32_t w = w0 + lane;
    const uint64_t rw = w < W ? row[w] : 0ull;
    const uint32_t c = (uint32_t)__popcll(rw);
    uint32_t x = c;  // exclusive prefix of c over the lanes
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    const uint32_t tot = (uint32_t)__shfl((int)x, 63, 64);
    uint32_t pos = cnt + x - c;
    for (uint64_t m = rw; m; m &= m - 1, ++pos) {
      const uint32_t j = w * 64 + (uint32_t)__builtin_ctzll(m);
      if (pos < CL_MMAX) {
        const QTd b = q[j];
        const float ex = qi.tx - b.tx, ey = qi.ty - b.ty, ez = qi.tz - b.tz;
        float d2 = 0.0f;
        d2 += ex * ex;
        d2 += ey * ey;
        d2 += ez * ez;
        key[pos] = ((uint64_t)__float_as_uint(d2) << 32) | j;
      }
    }
    cnt += tot;
  }
  if (cnt > CL_MMAX) {  // the host redoes this type
    if (lane == 0) stat[0] = 2;
    return;
  }
  // bitonic sort of key[0..cnt) (padded to a power of two with the max key)
  uint32_t P2 = 1;
  while (P2 < cnt) P2 <<= 1;
  for (uint32_t p = cnt + lane; p < P2; p += 64) key[p] = ~0ull;
  wsync();
  for (uint32_t s = 2; s <= P2; s <<= 1)
    for (uint32_t d = s >> 1; d > 0; d >>= 1) {
      for (uint32_t p = lane; p < P2; p += 64) {
        const uint32_t o = p ^ d;
        if (o > p) {
          const uint64_t a = key[p], b = key[o];
          const bool up = (p & s) == 0;
          if ((a > b) == up) {
            key[p] = b;
            key[o] = a;
          }
        }
      }
      wsync();
    }
  // members' records in (d2, j) order, then the sums in that order by one lane
  for (uint32_t p = lane; p < cnt; p += 64) {
    const QTd b = q[(uint32_t)key[p]];
    mtx[p] = b.tx;
    mty[p] = b.ty;
    mtz[p] = b.tz;
    mq[p][0] = b.qw;
    mq[p][1] = b.qx;
    mq[p][2] = b.qy;
    mq[p][3] = b.qz;
  }
  wsync();
  if (lane != 0) return;
  float ax = 0, ay = 0, az = 0;
  for (uint32_t p = 0; p < cnt; ++p) {
    ax = ax + mtx[p];
    ay = ay + mty[p];
    az = az + mtz[p];
  }
  const float cs = (float)cnt;
  ax = ax / cs;
  ay = ay / cs;
  az = az / cs;
  float s1[3] = {0, 0, 0}, s2[3] = {0, 0, 0};
  for (uint32_t p = 0; p < cnt; ++p) {
    const quatf qq = {mq[p][0], mq[p][1], mq[p][2], mq[p][3]};
    const f3 u = quat_rotate(qq, f3{1.f, 0.f, 0.f}), v = quat_rotate(qq, f3{0.f, 1.f, 0.f});
    s1[0] = s1[0] + u.x; s1[1] = s1[1] + u.y; s1[2] = s1[2] + u.z;
    s2[0] = s2[0] + v.x; s2[1] = s2[1] + v.y; s2[2] = s2[2] + v.z;
  }
  const f3 nt1 = normalize3(f3{s1[0] / cs, s1[1] / cs, s1[2] / cs});
  const f3 nt2 = normalize3(f3{s2[0] / cs, s2[1] / cs, s2[2] / cs});
  const quatf r = quat_from_rot(axes_to_rot(nt1, nt2));
  out.fine[(size_t)t * out.fcap + e] = QTd{r.w, r.x, r.y, r.z, ax, ay, az, 1u};
}

}  // namespace

void cluster_device(const ClusterIn& in, const ClusterOut& out, hipStream_t st) {
  k_cluster_seeds<<<3, 64, 0, st>>>(in, out);
  k_cluster_avg<<<dim3(out.egrid, 3), 64, 0, st>>>(in, out);
}

}  // namespace fccf
