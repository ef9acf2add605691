// match.hip — K5: all-pairs coplane-pair correspondence search (FCCF.cpp:1410-1428)
// fused with the closed-form transform of each match (computer_transform, :841-1018).
//
// One wave per test k = i1 * B2 + i2 (b1-major, the reference loop order).  A test
// passes when |angle1 - angle2| < 5 deg and the roughness types agree; it then emits
// one transform per (third source plane, matching target plane) in loop order, or
// the weighted-centroid fallback (:1000-1017).  Emission is two-pass: counts ->
// per-type exclusive scan -> write, so each type's list is in exactly the order
// transformation_vecter[type] receives push_backs.  The plane/pair tables (<= 16
// planes, <= 120 pairs per cloud) live in LDS.
#define KT_TU 6  // ktrace.h source tag
#include "probe.h"
#include "kernels.h"
#include "match.h"
#include "mail.h"

namespace fccf {
namespace {

struct Ctx {
  m33 rot;
  f3 n1, m1, n2, m2r, n1cm1, n2cm2;
};

__device__ void prep(const MatchIn& M, int i11, int i12, int i21, int i22, Ctx& c) {
  const MPlane *A = M.F1, *B = M.F2;
  c.n1 = {A[i11].n[0], A[i11].n[1], A[i11].n[2]};
  c.m1 = {A[i12].n[0], A[i12].n[1], A[i12].n[2]};
  c.n2 = {B[i21].n[0], B[i21].n[1], B[i21].n[2]};
  f3 m2 = {B[i22].n[0], B[i22].n[1], B[i22].n[2]};
  const f3 r1 = normalize3(cross3(c.n2, c.n1));
  const float n2dn1 = dot3(c.n2, c.n1);
  const float r1cn2dn1 = dot3(cross3(r1, c.n2), c.n1);
  const m33 R1 = rodrigues(n2dn1, r1cn2dn1, r1);
  m2 = mul3v(R1, m2);
  const f3 r2 = c.n1;
  const float m2dm1 = dot3(m2, c.m1), m2dr2 = dot3(m2, r2), m1dr2 = dot3(c.m1, r2);
  const float r2cm2dm1 = dot3(cross3(r2, m2), c.m1);
  const float cos2 = (m2dm1 - (m2dr2 * m1dr2)) / (1.f - (m2dr2 * m1dr2));
  const float sin2 = (r2cm2dm1) / (1.f - (m2dr2 * m1dr2));
  c.rot = mul33(rodrigues(cos2, sin2, r2), R1);
  c.m2r = m2;
  c.n1cm1 = normalize3(cross3(c.n1, c.m1));
  c.n2cm2 = normalize3(cross3(c.n2, m2));
}

__device__ __forceinline__ m44 rot_only(const m33& R) {
  m44 T = eye44();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
  return T;
}

// ((A^T A)^-1 A^T) D with Eigen's 3x3 cofactor inverse (compute_inverse<...,3>).
__device__ f3 ls3(f3 n1, f3 m1, f3 k1, f3 D) {
  m33 A, AT;
  const f3 rows[3] = {n1, m1, k1};
  for (int i = 0; i < 3; ++i) {
    A.m[i][0] = rows[i].x; A.m[i][1] = rows[i].y; A.m[i][2] = rows[i].z;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) AT.m[i][j] = A.m[j][i];
  const m33 M = mul33(AT, A);
#define COF(i, j) (M.m[((i) + 1) % 3][((j) + 1) % 3] * M.m[((i) + 2) % 3][((j) + 2) % 3] - \
                   M.m[((i) + 1) % 3][((j) + 2) % 3] * M.m[((i) + 2) % 3][((j) + 1) % 3])
  const float c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
  const float det = c0 * M.m[0][0] + (c1 * M.m[1][0] + c2 * M.m[2][0]);
  const float inv = 1.f / det;
  m33 Mi;
  Mi.m[0][0] = c0 * inv; Mi.m[0][1] = c1 * inv; Mi.m[0][2] = c2 * inv;
  Mi.m[1][0] = COF(0, 1) * inv; Mi.m[1][1] = COF(1, 1) * inv; Mi.m[1][2] = COF(2, 1) * inv;
  Mi.m[2][0] = COF(0, 2) * inv; Mi.m[2][1] = COF(1, 2) * inv; Mi.m[2][2] = COF(2, 2) * inv;
#undef COF
  return mul3v(mul33(Mi, AT), D);
}

// One wave per test k = i1 * B2 + i2.  Its candidate (third source plane k3,
// target plane q) pairs, p = k3 * nF2 + q in the reference's loop order, are spread
// over the lanes; ballot + mbcnt give every accepted pair its rank, so emission
// keeps loop order.  Returns the number of transforms the test emits (>= 1 when
// the test passes: the weighted-centroid fallback); writes them when out != null.
// hq (may be null): host mailbox of this type; qout[r] goes to hq[hoff + r] too while in capacity.
__device__ int match_test_wave(const MatchIn& M, int k, MCand* out, QTd* qout, QTd* hq = nullptr, uint32_t hoff = 0) {
  const int lane = threadIdx.x & 63;
  const int i1 = k / M.nB2, i2 = k % M.nB2;
  const MBase& b1 = M.B1[i1];
  const MBase& b2 = M.B2[i2];
  if (!(fabsf(b1.angle - b2.angle) < M.ang_same && b1.type == b2.type)) return 0;
  Ctx c;
  prep(M, b1.i1, b1.i2, b2.i1, b2.i2, c);
  const m44 T0 = rot_only(c.rot);
  const quatf qr = quat_from_rot(c.rot);  // fused R -> quaternion (FCCF.cpp:1437-1462)
  const MPlane *A = M.F1, *B = M.F2;
  const int np = M.nF1 * M.nF2;
  int cnt = 0;
  for (int p0 = 0; p0 < np; p0 += 64) {
    const int p = p0 + lane;
    bool ok = false;
    int k3 = 0, q = 0;
    f3 kn = {0.f, 0.f, 0.f}, pn = {0.f, 0.f, 0.f};
    if (p < np) {
      k3 = p / M.nF2;
      q = p % M.nF2;
      kn = {A[k3].n[0], A[k3].n[1], A[k3].n[2]};
      if (k3 != b1.i1 && k3 != b1.i2 && q != b2.i1 && q != b2.i2 && fabsf(dot3(c.n1cm1, kn)) > M.third_thr) {
        pn = tf_so3(T0, B[q].n[0], B[q].n[1], B[q].n[2]);
        ok = angle_lt(normal_cos(kn, pn), M.third_cut) && fabsf(dot3(c.n2cm2, pn)) > M.third_thr;
      }
    }
    const uint64_t m = __ballot(ok);
    if (out && ok) {
      const int r = cnt + (int)__popcll(m & ((1ull << lane) - 1ull));
      const f3 pc = tf_se3(T0, B[q].c[0], B[q].c[1], B[q].c[2]);
      const f3 c11 = {A[b1.i1].c[0], A[b1.i1].c[1], A[b1.i1].c[2]};
      const f3 c12 = {A[b1.i2].c[0], A[b1.i2].c[1], A[b1.i2].c[2]};
      const f3 c13 = {A[k3].c[0], A[k3].c[1], A[k3].c[2]};
      const f3 c21 = {B[b2.i1].c[0], B[b2.i1].c[1], B[b2.i1].c[2]};
      const f3 c22 = {B[b2.i2].c[0], B[b2.i2].c[1], B[b2.i2].c[2]};
      const f3 D = {dot3(c11, c.n1) - dot3(c21, c.n2), dot3(c12, c.m1) - dot3(c22, c.m2r),
                    dot3(c13, kn) - dot3(pc, pn)};
      const f3 t = ls3(c.n1, c.m1, kn, D);
      MCand& o = out[r];
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) o.R[3 * a + b] = c.rot.m[a][b];
      o.t[0] = t.x; o.t[1] = t.y; o.t[2] = t.z;
      const QTd qv = {qr.w, qr.x, qr.y, qr.z, t.x, t.y, t.z, 0u};
      qout[r] = qv;
      if (hq && hoff + (uint32_t)r < MatchMail::Q_CAP) hq[hoff + r] = qv;
    }
    cnt += (int)__popcll(m);
  }
  if (cnt == 0) {
    if (out && lane == 0) {
      const MPlane &a = A[b1.i1], &b = A[b1.i2], &d = B[b2.i1], &e = B[b2.i2];
      const float sx = (a.c[0] * a.fps + b.c[0] * b.fps) / (a.fps + b.fps);
      const float sy = (a.c[1] * a.fps + b.c[1] * b.fps) / (a.fps + b.fps);
      const float sz = (a.c[2] * a.fps + b.c[2] * b.fps) / (a.fps + b.fps);
      const float tx = (d.c[0] * d.fps + e.c[0] * e.fps) / (d.fps + e.fps);
      const float ty = (d.c[1] * d.fps + e.c[1] * e.fps) / (d.fps + e.fps);
      const float tz = (d.c[2] * d.fps + e.c[2] * e.fps) / (d.fps + e.fps);
      const f3 tc = mul3v(c.rot, f3{tx, ty, tz});
      MCand& o = out[0];
      for (int a2 = 0; a2 < 3; ++a2)
        for (int b2i = 0; b2i < 3; ++b2i) o.R[3 * a2 + b2i] = c.rot.m[a2][b2i];
      o.t[0] = sx - tc.x; o.t[1] = sy - tc.y; o.t[2] = sz - tc.z;
      const QTd qv = {qr.w, qr.x, qr.y, qr.z, o.t[0], o.t[1], o.t[2], 0u};
      qout[0] = qv;
      if (hq && hoff < MatchMail::Q_CAP) hq[hoff] = qv;
    }
    cnt = 1;
  }
  return cnt;
}

// The plane/pair tables into LDS, all threads copying 16-byte words.
__device__ __forceinline__ void load_tables(MatchIn& M, const MatchIn* __restrict__ Mp) {
  static_assert(sizeof(MatchIn) % 16 == 0, "MatchIn is copied in 16-byte words");
  const int4* src = reinterpret_cast<const int4*>(Mp);
  int4* dst = reinterpret_cast<int4*>(&M);
  for (int i = threadIdx.x; i < (int)(sizeof(MatchIn) / 16); i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

__global__ void __launch_bounds__(256) k_match_count(const MatchIn* __restrict__ Mp, uint32_t* __restrict__ cnt,
                                                     int32_t* __restrict__ type) {
  KT();
  __shared__ __attribute__((aligned(16))) MatchIn M;
  load_tables(M, Mp);
  const int K = M.nB1 * M.nB2;
  for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < K; k += gridDim.x * 4) {
    const int n = match_test_wave(M, k, nullptr, nullptr);
    if ((threadIdx.x & 63) == 0) {
      cnt[k] = (uint32_t)n;
      type[k] = n ? M.B1[k / M.nB2].type : -1;
    }
  }
}

// single block of 1024 threads: per-type exclusive scan in test order.  Thread t
// owns a contiguous run of tests: local per-type sums, one block scan of the
// three sums, then a second walk over its run writes the offsets.
__global__ void __launch_bounds__(1024) k_match_scan(const MatchIn* __restrict__ Mp, const uint32_t* __restrict__ cnt,
                                                     const int32_t* __restrict__ type, uint32_t* __restrict__ off,
                                                     uint32_t* __restrict__ totals, MatchMail* __restrict__ mail) {
  KT();
  __shared__ uint32_t sh[16][3];
  __shared__ uint32_t kp;
  if (threadIdx.x == 0) kp = 0;
  const int K = Mp->nB1 * Mp->nB2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = (K + 1023) / 1024;
  const int k0 = min(K, (int)threadIdx.x * per), k1 = min(K, k0 + per);
  uint32_t loc[3] = {0, 0, 0}, pass = 0;
  for (int k = k0; k < k1; ++k) {
    const int t = type[k];
    const uint32_t c = cnt[k];
    loc[0] += t == 0 ? c : 0u;
    loc[1] += t == 1 ? c : 0u;
    loc[2] += t == 2 ? c : 0u;
    pass += c ? 1u : 0u;
  }
  uint32_t inc[3];
#pragma unroll
  for (int ty = 0; ty < 3; ++ty) {
    uint32_t x = loc[ty];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    inc[ty] = x;
    if (lane == 63) sh[w][ty] = x;
  }
  __syncthreads();
  uint32_t run[3];
#pragma unroll
  for (int ty = 0; ty < 3; ++ty) {
    uint32_t wp = 0, tot = 0;
    for (int ww = 0; ww < 16; ++ww) {
      wp += ww < w ? sh[ww][ty] : 0u;
      tot += sh[ww][ty];
    }
    run[ty] = wp + inc[ty] - loc[ty];
    if (threadIdx.x == 0) {
      totals[ty] = tot;
      if (mail) mail->tot[ty] = tot;
    }
  }
  if (mail) {  // K_pass for the stats (tests with >= 1 candidate)
    if (pass) atomicAdd(&kp, pass);
    __syncthreads();
    if (threadIdx.x == 0) mail->kpass = kp;
  }
  for (int k = k0; k < k1; ++k) {
    const int t = type[k];
    const uint32_t c = cnt[k];
    uint32_t o = 0;
#pragma unroll
    for (int ty = 0; ty < 3; ++ty)
      if (t == ty) {
        o = run[ty];
        run[ty] += c;
      }
    off[k] = o;
  }
}

#ifndef EMIT_WPE
#define EMIT_WPE 1
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EMIT_WPE))) k_match_emit(const MatchIn* __restrict__ Mp, const uint32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ type, const uint32_t* __restrict__ off,
                                                    MCand* __restrict__ c0, MCand* __restrict__ c1,
                                                    MCand* __restrict__ c2, QTd* __restrict__ q0,
                                                    QTd* __restrict__ q1, QTd* __restrict__ q2,
                                                    MatchMail* __restrict__ mail) {
  KT();
  __shared__ __attribute__((aligned(16))) MatchIn M;
  load_tables(M, Mp);
  const int K = M.nB1 * M.nB2;
  for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < K; k += gridDim.x * 4) {
    if (!cnt[k]) continue;
    const int t = type[k];
    MCand* cb = t == 0 ? c0 : (t == 1 ? c1 : c2);
    QTd* qb = t == 0 ? q0 : (t == 1 ? q1 : q2);
    const uint32_t o = off[k];
    match_test_wave(M, k, cb + o, qb + o, mail ? mail->q[t] : nullptr, o);
  }
}

// transform_cluster's radius search (FCCF.cpp:1075-1103) as a bitmask: bit j of
// row i is set when candidate j is a neighbour of seed i, i.e. d2 < r^2 (the
// FLANN L2_Simple sum ((0 + ex^2) + ey^2) + ez^2) and the x axes of the two
// rotations are within the cluster angle.  Which candidates a seed takes does not
// depend on earlier seeds (every neighbour is pushed), so all rows are
// independent; the host applies them in seed order (host_stages.cpp).  One wave
// per (row, 64-column word): lane = column, the ballot is the word, written
// straight into the pinned mailbox.  Rows of candidates with a non-finite tx come
// out empty (d2 is NaN or inf), as in the host path.
__global__ void __launch_bounds__(256) k_cluster_bits(const QTd* __restrict__ q0, const QTd* __restrict__ q1,
                                                      const QTd* __restrict__ q2, const uint32_t* __restrict__ totals,
                                                      float r2, AngleCut ccut, float min_n, uint64_t* __restrict__ out,
                                                      uint64_t* __restrict__ dout) {
  KT();
  const int t = blockIdx.y;
  const QTd* __restrict__ q = t == 0 ? q0 : (t == 1 ? q1 : q2);
  uint64_t words = 0, off = 0;
  for (int u = 0; u < 3; ++u) {
    const uint64_t n = totals[u], w = ((n + 63) / 64) * n;
    if (u < t) off += w;
    words += w;
  }
  if (words > MatchMail::CB_CAP) return;  // the host falls back to its own search
  const uint32_t n = totals[t];
  if ((float)n <= min_n) return;  // cluster_number_threshold: not clustered
  const uint32_t W = (n + 63) / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t ntask = (uint64_t)n * W;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < ntask; g += (uint64_t)gridDim.x * 4) {
    const uint32_t i = (uint32_t)(g / W), w = (uint32_t)(g % W);
    const uint32_t j = w * 64 + lane;
    const QTd a = q[i];
    bool nb = false;
    if (j < n) {
      const QTd b = q[j];
      const float ex = a.tx - b.tx, ey = a.ty - b.ty, ez = a.tz - b.tz;
      float d2 = 0.0f;
      d2 += ex * ex;
      d2 += ey * ey;
      d2 += ez * ez;
      if (d2 < r2) {
        const f3 xa = quat_rotate(quatf{a.qw, a.qx, a.qy, a.qz}, f3{1.f, 0.f, 0.f});
        const f3 xb = quat_rotate(quatf{b.qw, b.qx, b.qy, b.qz}, f3{1.f, 0.f, 0.f});
        nb = angle_lt(normal_cos(xa.x, xa.y, xa.z, xb.x, xb.y, xb.z), ccut);
      }
    }
    const uint64_t m = __ballot(nb);
    if (lane == 0) {
      out[off + g] = m;
      if (dout) dout[off + g] = m;
    }
  }
}

}  // namespace

void match_candidates(const MatchIn* d_in, int K, uint32_t* cnt, int32_t* type, uint32_t* off, uint32_t* totals,
                      MCand* c[3], QTd* q[3], hipStream_t st, MatchMail* mail) {
  if (K <= 0) return;
  const int g = (K + 3) / 4;  // one wave per test
  FCCF_LAUNCH("k_match_count", (nullptr, 0.0, nullptr, 0.0, (double)sizeof(MatchIn)), k_match_count, g, 256, 0, st, d_in, cnt, type);
  k_match_scan<<<1, 1024, 0, st>>>(d_in, cnt, type, off, totals, mail);
  FCCF_LAUNCH("k_match_emit", (nullptr, 0.0, nullptr, 0.0, (double)sizeof(MatchIn)), k_match_emit, g, 256, 0, st, d_in, cnt, type, off, c[0], c[1], c[2], q[0], q[1], q[2], mail);
}

void cluster_bits(QTd* const q[3], const uint32_t* totals, float r2, AngleCut ccut, float min_n, MatchMail* mail,
                  hipStream_t st, uint64_t* dev_rows) {
  k_cluster_bits<<<dim3(512, 3), 256, 0, st>>>(q[0], q[1], q[2], totals, r2, ccut, min_n, mail->cbits, dev_rows);
}

}  // namespace fccf
