// rn_bn.hip -- BatchNorm (+ fused ReLU) forward / backward on NHWC activations.
//
// Replaces mx.sym.BatchNorm followed by mx.sym.Activation(act_type='relu') of the reference
// graphs (symbol/resnet.py:12-23,90-96,111-112; symbol/resnext.py:20-46). Training semantics
// (MXNet 1.x, restated in oracle/ops.py): batch mean / biased variance over N*H*W,
// moving = moving*momentum + batch*(1-momentum), fix_gamma => gamma := 1 and dgamma := 0.
//
// HBM-bound: every pass reads each element once with 16-byte (8 x bf16) loads.
//  fwd : stats pass (per-block shifted sums) -> finalize (fp64 combine) -> apply(+relu) pass
//  bwd : reduce pass (sum dz, sum dz*(x-mean)) -> finalize -> apply pass (+ optional add_src)
// Workspace layout (floats): partials[nrb][c][2] | coef[c][4]
#include <algorithm>

#include "rn_common.h"

// 16-byte chunk loads / stores of the streaming BatchNorm passes, NT = rn_set_tuning 18 bit mask:
// 1 = nontemporal stores, 2 = nontemporal loads (the streaming hint: lines are evicted first, so
// fewer dirty lines are left for the kernel-boundary L2 write-back and the other stream's tiles keep
// their L2 share); 4 = write-through stores instead (the apply passes with rn_set_tuning 18 bit 32).
typedef unsigned int rn_u32x4 __attribute__((ext_vector_type(4)));
template <int NT>
__device__ __forceinline__ uint4 ld16(const void* p) {
  if constexpr ((NT & 2) != 0) {
    const rn_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const rn_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}
template <int NT>
__device__ __forceinline__ void st16(void* p, uint4 v) {
  if constexpr ((NT & 4) != 0) {
    // write-through (sc1): the line leaves no dirty copy in the XCD's L2 for the end-of-kernel write-back
    // (rn_set_tuning 18 bit 32). Asm the compiler does not see: the nop keeps its next instruction off the
    // data registers until the store has read them
    const rn_u32x4 w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr ((NT & 1) != 0) {
    const rn_u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<rn_u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}
// bit 4: the reduction / residual-tail read passes (bn_bwd_reduce, relu_bwd_bnred, bn_add) load
// with the same hint
inline bool nt_reads() { return (g_tune[RN_TUNE_BN_NT] & 6) == 6; }

namespace {

constexpr int kThreads = 256;

struct Geo {
  int cpr;   // chunks per row
  int ct;    // chunk lanes per block (divides cpr or == cpr)
  int rl;    // row lanes per block
  int gx;    // blocks along channels
  int nrb;   // blocks along rows
  int64_t rows_per_block;
};

template <typename T>
Geo make_geo(int64_t m, int c) {
  Geo g;
  const int CE = 16 / sizeof(T);
  g.cpr = c / CE;
  g.ct = std::min(g.cpr, 32);
  while (g.cpr % g.ct) --g.ct;
  g.rl = kThreads / g.ct;
  g.gx = g.cpr / g.ct;
  int64_t want = std::max<int64_t>(1, 2048 / g.gx);
  int64_t maxrb = std::max<int64_t>(1, m / (g.rl * 4));
  g.nrb = (int)std::min(want, maxrb);
  g.rows_per_block = ceil_div(m, g.nrb);
  return g;
}

__device__ __forceinline__ float relu_mask(float x, float sc, float sh) { return fmaf(x, sc, sh) > 0.f ? 1.f : 0.f; }
// the backward's dz mask with a folded Quantization_int8 straight-through clip (rn_bn_desc.clip): the
// ReLU, and zero where the output as stored (rounded to T, as bn_apply_kernel writes it) is >= t
template <typename T>
__device__ __forceinline__ float relu_clip_mask(float x, float sc, float sh, bool clip, float t) {
  const float z = fmaf(x, sc, sh);
  return (z > 0.f && (!clip || to_f(from_f<T>(z)) < t)) ? 1.f : 0.f;
}

// the dz of a BatchNorm+ReLU whose output two Quantization_int8 read (rn_bn_desc.dy2): both
// straight-through backwards summed and rounded to T, as two rn_quant_int8_bwd calls store them
template <typename T>
__device__ __forceinline__ float relu_clip2_dz(float x, float sc, float sh, float g1, float t1, float g2, float t2) {
  const float z = fmaf(x, sc, sh);
  if (!(z > 0.f)) return 0.f;
  const float y = to_f(from_f<T>(z));
  return to_f(from_f<T>((y < t1 ? g1 : 0.f) + (y < t2 ? g2 : 0.f)));
}

// ---- forward stats: partial shifted sums; pivot = x[0][c]
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* __restrict__ x, int64_t m, int c, int ct,
                                                       int64_t rows_per_block, float* __restrict__ part) {
  constexpr int CE = 16 / sizeof(T);
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cbase = (blockIdx.x * ct + tc) * CE;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float piv[CE], s[CE], q[CE];
  {
    uint4 u = *reinterpret_cast<const uint4*>(x + cbase);
    chunk_to_f(u, piv, (const T*)nullptr);
  }
#pragma unroll
  for (int e = 0; e < CE; ++e) s[e] = q[e] = 0.f;
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    uint4 u = *reinterpret_cast<const uint4*>(x + r * c + cbase);
    float f[CE];
    chunk_to_f(u, f, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const float d = f[e] - piv[e];
      s[e] += d;
      q[e] = fmaf(d, d, q[e]);
    }
  }
  __shared__ float red[kThreads * (8 * 2 + 1)];  // odd row stride: conflict-free LDS writes
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    red[(tr * ct + tc) * (CE * 2 + 1) + 2 * e] = s[e];
    red[(tr * ct + tc) * (CE * 2 + 1) + 2 * e + 1] = q[e];
  }
  __syncthreads();
  // reduce over row lanes: thread t < ct*CE*2 sums column t
  const int ncol = ct * CE * 2;
  for (int col = threadIdx.x; col < ncol; col += blockDim.x) {
    float acc = 0.f;
    const int tcv = col / (CE * 2), v = col - tcv * (CE * 2);
    for (int r = 0; r < rl; ++r) acc += red[(r * ct + tcv) * (CE * 2 + 1) + v];
    const int cc = blockIdx.x * ct * CE + col / 2;
    part[((int64_t)blockIdx.y * c + cc) * 2 + (col & 1)] = acc;
  }
}

// finalize: one block per channel; fp64 reduction of the per-row-block partials.
__device__ __forceinline__ void block_sum2(double& s, double& q) {
  __shared__ double rs[256], rq[256];
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      rs[threadIdx.x] += rs[threadIdx.x + o];
      rq[threadIdx.x] += rq[threadIdx.x + o];
    }
    __syncthreads();
  }
  s = rs[0];
  q = rq[0];
}

template <typename T>
__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const T* __restrict__ x, const float* __restrict__ part,
                                                              int nrb, int64_t m, int c, int c_real, float eps,
                                                              float momentum, int fix_gamma,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* moving_mean,
                                                              float* moving_var, float* save_mean, float* save_invstd,
                                                              float* scale, float* shift) {
  const int ch = blockIdx.x;
  double s = 0.0, q = 0.0;
  for (int b = threadIdx.x; b < nrb; b += blockDim.x) {
    const float2 v = reinterpret_cast<const float2*>(part)[(int64_t)b * c + ch];
    s += v.x;
    q += v.y;
  }
  block_sum2(s, q);
  if (threadIdx.x != 0) return;
  if (ch >= c_real) {
    scale[ch] = 0.f;
    shift[ch] = 0.f;
    return;
  }
  const double piv = (double)to_f(x[ch]);
  const double md = s / (double)m;
  const double mean = piv + md;
  double var = q / (double)m - md * md;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = fix_gamma ? 1.f : gamma[ch];
  const float sc = g * invstd;
  scale[ch] = sc;
  shift[ch] = beta[ch] - (float)mean * sc;
  save_mean[ch] = (float)mean;
  save_invstd[ch] = invstd;
  if (moving_mean) {
    moving_mean[ch] = moving_mean[ch] * momentum + (float)mean * (1.f - momentum);
    moving_var[ch] = moving_var[ch] * momentum + (float)var * (1.f - momentum);
  }
}

// finalize from per-row-block partials written by a producing kernel's epilogue (the conv
// epilogue of rn_conv_fwd_bnstats): part[b][0|1|2][ld] = S1 = sum(v - p_b), S2 = sum((v - p_b)^2)
// and the pivot p_b, over the block's n_b rows. Shifting a partial to another pivot q is exact:
//   S1' = S1 + n d,  S2' = S2 + 2 d S1 + n d^2,  d = p_b - q.
// Pass 1 (grid c/64 x groups of 64 row blocks, reads coalesced across channels) merges each group
// onto its first pivot in fp64; pass 2 merges the groups per channel and finalizes.
constexpr int kPartGroup = 64;
__global__ __launch_bounds__(256) void bn_part_merge_kernel(const float* __restrict__ part, int nblk, int64_t m,
                                                            int rows_blk, int ld, int c,
                                                            double* __restrict__ part2) {
  const int ch = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;
  const int b0 = blockIdx.y * kPartGroup;
  const int b1 = min(nblk, b0 + kPartGroup);
  __shared__ double red[3][4][64];
  double s1 = 0.0, s2 = 0.0, n = 0.0, q = 0.0;
  if (ch < c) {
    q = part[(int64_t)b0 * 3 * ld + 2 * ld + ch];
    // every load of the group issued before the (same-order) fp64 sums: one memory latency, not 16
    constexpr int kPer = kPartGroup / 4;
    float va[kPer], vs[kPer], vp[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int b = b0 + sub + 4 * u;
      const float* pb = part + (int64_t)min(b, b1 - 1) * 3 * ld + ch;
      va[u] = pb[0];
      vs[u] = pb[ld];
      vp[u] = pb[2 * ld];
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int b = b0 + sub + 4 * u;
      if (b >= b1) break;
      const double nb = (double)min<int64_t>(rows_blk, m - (int64_t)b * rows_blk);
      const double d = (double)vp[u] - q;
      const double a = va[u];
      s1 += a + nb * d;
      s2 += (double)vs[u] + 2.0 * d * a + nb * d * d;
      n += nb;
    }
  }
  red[0][sub][threadIdx.x & 63] = s1;
  red[1][sub][threadIdx.x & 63] = s2;
  red[2][sub][threadIdx.x & 63] = n;
  __syncthreads();
  if (sub == 0 && ch < c) {
    for (int t = 1; t < 4; ++t) {
      s1 += red[0][t][threadIdx.x];
      s2 += red[1][t][threadIdx.x];
      n += red[2][t][threadIdx.x];
    }
    double* dst = part2 + (int64_t)blockIdx.y * 4 * c + ch;
    dst[0] = s1;
    dst[c] = s2;
    dst[2 * c] = n;
    dst[3 * c] = q;
  }
}

__global__ __launch_bounds__(256) void bn_fwd_finalize_part_kernel(const double* __restrict__ part2, int ngrp,
                                                                   int64_t m, int c, int c_real, float eps,
                                                                   float momentum, int fix_gamma,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta,
                                                                   float* moving_mean, float* moving_var,
                                                                   float* save_mean, float* save_invstd,
                                                                   float* scale, float* shift) {
  // 4 threads per channel walk the groups (latency-bound loop: more of them in flight), then an LDS sum
  const int ch = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;
  __shared__ double red[2][4][64];
  double s1 = 0.0, s2 = 0.0, q = 0.0;
  if (ch < c) {
    q = part2[3 * c + ch];  // group 0's pivot
    for (int g0 = sub; g0 < ngrp; g0 += 16) {  // 4 groups' loads in flight, summed in group order
      double va[4], vs[4], vn[4], vp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double* pg = part2 + (int64_t)min(g0 + 4 * u, ngrp - 1) * 4 * c + ch;
        va[u] = pg[0];
        vs[u] = pg[c];
        vn[u] = pg[2 * c];
        vp[u] = pg[3 * c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (g0 + 4 * u >= ngrp) break;
        const double d = vp[u] - q, a = va[u], nb = vn[u];
        s1 += a + nb * d;
        s2 += vs[u] + 2.0 * d * a + nb * d * d;
      }
    }
  }
  red[0][sub][threadIdx.x & 63] = s1;
  red[1][sub][threadIdx.x & 63] = s2;
  __syncthreads();
  if (sub != 0 || ch >= c) return;
  for (int t = 1; t < 4; ++t) {
    s1 += red[0][t][threadIdx.x];
    s2 += red[1][t][threadIdx.x];
  }
  if (ch >= c_real) {
    scale[ch] = 0.f;
    shift[ch] = 0.f;
    return;
  }
  const double md = s1 / (double)m;
  const double mean = q + md;
  double var = s2 / (double)m - md * md;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = fix_gamma ? 1.f : gamma[ch];
  const float sc = g * invstd;
  scale[ch] = sc;
  shift[ch] = beta[ch] - (float)mean * sc;
  save_mean[ch] = (float)mean;
  save_invstd[ch] = invstd;
  if (moving_mean) {
    moving_mean[ch] = moving_mean[ch] * momentum + (float)mean * (1.f - momentum);
    moving_var[ch] = moving_var[ch] * momentum + (float)var * (1.f - momentum);
  }
}

// bn_part_merge_kernel + bn_fwd_finalize_part_kernel in ONE launch where the partials form at most 4
// merge groups (nblk <= 4 * kPartGroup: the stage-3/4 layers' 224-row conv tiles, ResNet-50 at batch 256).
// A block takes 16 channels; thread (group g, sub v, channel) forms the merge kernel's sub-sum v of group g
// (its 16 interleaved blocks -- every load of it in flight at once, as there), the four sub-sums of a group
// are added in sub order, then the finalize kernel's walk over the groups in group order: outputs
// bit-identical to the two launches, one launch and one kernel boundary fewer on the forward chain
__global__ __launch_bounds__(256) void bn_fwd_merge_finalize_kernel(
    const float* __restrict__ part, int nblk, int64_t m, int rows_blk, int ld, int c, int c_real, float eps,
    float momentum, int fix_gamma, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* moving_mean, float* moving_var, float* save_mean, float* save_invstd, float* scale, float* shift) {
  const int cl = threadIdx.x & 15, ch = blockIdx.x * 16 + cl;
  const int g = threadIdx.x >> 6, v = (threadIdx.x >> 4) & 3;
  const int ngrp = (nblk + kPartGroup - 1) / kPartGroup;
  __shared__ double sub[3][4][4][16];  // [s1, s2, n][group][sub][channel]
  __shared__ double piv[4][16];
  if (ch < c && g < ngrp) {
    const int b0 = g * kPartGroup, b1 = min(nblk, b0 + kPartGroup);
    const double q = part[(int64_t)b0 * 3 * ld + 2 * ld + ch];
    constexpr int kPer = kPartGroup / 4;
    float va[kPer], vs[kPer], vp[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int b = b0 + v + 4 * u;
      const float* pb = part + (int64_t)min(b, b1 - 1) * 3 * ld + ch;
      va[u] = pb[0];
      vs[u] = pb[ld];
      vp[u] = pb[2 * ld];
    }
    double s1 = 0.0, s2 = 0.0, n = 0.0;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int b = b0 + v + 4 * u;
      if (b >= b1) break;
      const double nb = (double)min<int64_t>(rows_blk, m - (int64_t)b * rows_blk);
      const double d = (double)vp[u] - q;
      const double a = va[u];
      s1 += a + nb * d;
      s2 += (double)vs[u] + 2.0 * d * a + nb * d * d;
      n += nb;
    }
    sub[0][g][v][cl] = s1;
    sub[1][g][v][cl] = s2;
    sub[2][g][v][cl] = n;
    if (v == 0) piv[g][cl] = q;
  }
  __syncthreads();
  if (threadIdx.x >= 16 || ch >= c) return;
  // per group: the merge kernel's sub sums in order; then the finalize kernel's per-sub terms (sub = group
  // here, each walking one group) added in group order
  const double q0 = piv[0][cl];
  double t1[4], t2[4];
#pragma unroll
  for (int gg = 0; gg < 4; ++gg) {
    t1[gg] = t2[gg] = 0.0;
    if (gg >= ngrp) continue;
    double a = sub[0][gg][0][cl], s = sub[1][gg][0][cl], nb = sub[2][gg][0][cl];
#pragma unroll
    for (int vv = 1; vv < 4; ++vv) {
      a += sub[0][gg][vv][cl];
      s += sub[1][gg][vv][cl];
      nb += sub[2][gg][vv][cl];
    }
    const double d = piv[gg][cl] - q0;
    t1[gg] += a + nb * d;
    t2[gg] += s + 2.0 * d * a + nb * d * d;
  }
  double s1 = t1[0], s2 = t2[0];
#pragma unroll
  for (int gg = 1; gg < 4; ++gg) {
    s1 += t1[gg];
    s2 += t2[gg];
  }
  if (ch >= c_real) {
    scale[ch] = 0.f;
    shift[ch] = 0.f;
    return;
  }
  const double md = s1 / (double)m;
  const double mean = q0 + md;
  double var = s2 / (double)m - md * md;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float gm = fix_gamma ? 1.f : gamma[ch];
  const float sc = gm * invstd;
  scale[ch] = sc;
  shift[ch] = beta[ch] - (float)mean * sc;
  save_mean[ch] = (float)mean;
  save_invstd[ch] = invstd;
  if (moving_mean) {
    moving_mean[ch] = moving_mean[ch] * momentum + (float)mean * (1.f - momentum);
    moving_var[ch] = moving_var[ch] * momentum + (float)var * (1.f - momentum);
  }
}

// ---- stem input (bn_data over the NCHW fp32 `data`, symbol/resnet.py:90): statistics straight from
// the NCHW planes, then one pass writing the normalised NHWC-8 compute copy for conv0.
// part[b][c][2]: shifted sums over images [b*ipb, (b+1)*ipb) of channel c, pivot x[0][c][0][0].
__global__ __launch_bounds__(256) void stem_stats_kernel(const float* __restrict__ x, int n, int c, int hw, int ipb,
                                                         float* __restrict__ part) {
  const int ch = blockIdx.x;
  const int b = blockIdx.y;
  const float piv = x[(int64_t)ch * hw];
  float s = 0.f, q = 0.f;
  for (int img = b * ipb; img < min(n, (b + 1) * ipb); ++img) {
    const float4* pl = reinterpret_cast<const float4*>(x + ((int64_t)img * c + ch) * hw);
    for (int i = threadIdx.x; i < hw / 4; i += blockDim.x) {
      const float4 v = pl[i];
      const float d0 = v.x - piv, d1 = v.y - piv, d2 = v.z - piv, d3 = v.w - piv;
      s += (d0 + d1) + (d2 + d3);
      q = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, q))));
    }
  }
  double sd = s, qd = q;
  block_sum2(sd, qd);
  if (threadIdx.x == 0) {
    part[((int64_t)b * c + ch) * 2] = (float)sd;
    part[((int64_t)b * c + ch) * 2 + 1] = (float)qd;
  }
}

__global__ __launch_bounds__(256) void stem_finalize_kernel(const float* __restrict__ x, const float* __restrict__ part,
                                                            int nb, int64_t m, int c, int hw, float eps,
                                                            float momentum, int fix_gamma, const float* gamma,
                                                            const float* beta, float* moving_mean, float* moving_var,
                                                            float* save_mean, float* save_invstd, float* scale,
                                                            float* shift) {
  const int ch = blockIdx.x;
  double s = 0.0, q = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    s += part[((int64_t)b * c + ch) * 2];
    q += part[((int64_t)b * c + ch) * 2 + 1];
  }
  block_sum2(s, q);
  if (threadIdx.x != 0) return;
  const double md = s / (double)m;
  const double mean = (double)x[(int64_t)ch * hw] + md;
  double var = q / (double)m - md * md;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = fix_gamma ? 1.f : gamma[ch];
  scale[ch] = g * invstd;
  shift[ch] = beta[ch] - (float)mean * g * invstd;
  save_mean[ch] = (float)mean;
  save_invstd[ch] = invstd;
  if (moving_mean) {
    moving_mean[ch] = moving_mean[ch] * momentum + (float)mean * (1.f - momentum);
    moving_var[ch] = moving_var[ch] * momentum + (float)var * (1.f - momentum);
  }
}

// thread per pixel: NCHW fp32 (c <= 8 channels) -> one 8-channel NHWC chunk, affine applied
template <typename T>
__global__ __launch_bounds__(256) void stem_to_nhwc8_kernel(const float* __restrict__ x, int64_t npix, int c, int hw,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, T* __restrict__ out) {
  constexpr int CE = 16 / sizeof(T);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i / hw;
    const int64_t pix = i - img * hw;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = 0.f;
      if (e < c) {
        f = x[(img * c + e) * hw + pix];
        if (scale) f = fmaf(f, scale[e], shift[e]);
      }
      v[e] = f;
    }
#pragma unroll
    for (int h = 0; h < 8 / CE; ++h)
      reinterpret_cast<uint4*>(out + i * 8)[h] = f_to_chunk(v + h * CE, (const T*)nullptr);
  }
}

__global__ void bn_infer_coef_kernel(int c, int c_real, float eps, int fix_gamma, const float* gamma,
                                     const float* beta, const float* mm, const float* mv, float* scale,
                                     float* shift) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  if (ch >= c_real) {
    scale[ch] = 0.f;
    shift[ch] = 0.f;
    return;
  }
  const float invstd = 1.f / sqrtf(mv[ch] + eps);
  const float g = fix_gamma ? 1.f : gamma[ch];
  scale[ch] = g * invstd;
  shift[ch] = beta[ch] - mm[ch] * g * invstd;
}

// 2D elementwise layout: thread (tc, tr) owns channel chunk blockIdx.x*ct+tc for rows
// blockIdx.y*rows_per_block + tr (step rl) -> per-channel coefficients live in registers.
template <typename T, bool RELU, int NT = 0>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int64_t m, int c, int ct,
                                                       int64_t rows_per_block) {
  constexpr int CE = 16 / sizeof(T);
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cbase = (blockIdx.x * ct + tc) * CE;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float sc[CE], sh[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    sc[e] = scale[cbase + e];
    sh[e] = shift[cbase + e];
  }
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    float f[CE];
    chunk_to_f(ld16<NT>(x + r * c + cbase), f, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const float v = fmaf(f[e], sc[e], sh[e]);
      f[e] = RELU ? fmaxf(v, 0.f) : v;
    }
    st16<NT>(y + r * c + cbase, f_to_chunk(f, (const T*)nullptr));
  }
}

// ---- post-activation unit tail (symbol/resnext.py:40-47, symbol/resnet.py:63-74): y = act(bn_a(xa) +
// b) with b = bn_b(xb) (the shortcut's BatchNorm) or xb itself. Each BatchNorm output is rounded to
// the storage type before the add, exactly as the unfused bn_apply + eltwise_add pair stores and
// re-reads it, so the result is bit-identical and the BatchNorm outputs are never written.
template <typename T, bool RELU, bool BNB, int NT = 0>
__global__ __launch_bounds__(256) void bn_add_kernel(const T* __restrict__ xa, const float* __restrict__ sca,
                                                     const float* __restrict__ sha, const T* __restrict__ xb,
                                                     const float* __restrict__ scb, const float* __restrict__ shb,
                                                     T* __restrict__ y, int64_t m, int c, int ct,
                                                     int64_t rows_per_block) {
  constexpr int CE = 16 / sizeof(T);
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cbase = (blockIdx.x * ct + tc) * CE;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float a_sc[CE], a_sh[CE], b_sc[BNB ? CE : 1], b_sh[BNB ? CE : 1];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    a_sc[e] = sca[cbase + e];
    a_sh[e] = sha[cbase + e];
    if constexpr (BNB) {
      b_sc[e] = scb[cbase + e];
      b_sh[e] = shb[cbase + e];
    }
  }
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    float fa[CE], fb[CE];
    chunk_to_f(ld16<NT>(xa + r * c + cbase), fa, (const T*)nullptr);
    chunk_to_f(ld16<NT>(xb + r * c + cbase), fb, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const float va = to_f(from_f<T>(fmaf(fa[e], a_sc[e], a_sh[e])));
      const float vb = BNB ? to_f(from_f<T>(fmaf(fb[e], b_sc[e], b_sh[e]))) : fb[e];
      const float v = va + vb;
      fa[e] = RELU ? fmaxf(v, 0.f) : v;
    }
    *reinterpret_cast<uint4*>(y + r * c + cbase) = f_to_chunk(fa, (const T*)nullptr);
  }
}

// ---- backward reduce: sum dz, sum dz*(x - mean)
template <typename T, bool RELU, bool PAIR = false, int NT = 0>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                            int64_t m, int c, int ct, int64_t rows_per_block,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            float* __restrict__ part,
                                                            const float* __restrict__ clip = nullptr,
                                                            const T* __restrict__ dy2 = nullptr,
                                                            const float* __restrict__ clip2 = nullptr) {
  constexpr int CE = 16 / sizeof(T);
  const bool hc = clip != nullptr;
  const float t = hc ? *clip : 0.f;
  const float t2 = PAIR ? *clip2 : 0.f;
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cbase = (blockIdx.x * ct + tc) * CE;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float mu[CE], sc[CE], sh[CE], s[CE], q[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    mu[e] = mean[cbase + e];
    sc[e] = scale[cbase + e];
    sh[e] = shift[cbase + e];
    s[e] = q[e] = 0.f;
  }
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    uint4 ux = ld16<NT>(x + r * c + cbase);
    uint4 ud = ld16<NT>(dy + r * c + cbase);
    float fx[CE], fd[CE], f2[CE];
    chunk_to_f(ux, fx, (const T*)nullptr);
    chunk_to_f(ud, fd, (const T*)nullptr);
    if constexpr (PAIR) chunk_to_f(ld16<NT>(dy2 + r * c + cbase), f2, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const float dz = PAIR ? relu_clip2_dz<T>(fx[e], sc[e], sh[e], fd[e], t, f2[e], t2)
                            : RELU ? fd[e] * relu_clip_mask<T>(fx[e], sc[e], sh[e], hc, t) : fd[e];
      s[e] += dz;
      q[e] = fmaf(dz, fx[e] - mu[e], q[e]);
    }
  }
  __shared__ float red[kThreads * (8 * 2 + 1)];  // odd row stride: conflict-free LDS writes
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    red[(tr * ct + tc) * (CE * 2 + 1) + 2 * e] = s[e];
    red[(tr * ct + tc) * (CE * 2 + 1) + 2 * e + 1] = q[e];
  }
  __syncthreads();
  const int ncol = ct * CE * 2;
  for (int col = threadIdx.x; col < ncol; col += blockDim.x) {
    float acc = 0.f;
    const int tcv = col / (CE * 2), v = col - tcv * (CE * 2);
    for (int r = 0; r < rl; ++r) acc += red[(r * ct + tcv) * (CE * 2 + 1) + v];
    const int cc = blockIdx.x * ct * CE + col / 2;
    part[((int64_t)blockIdx.y * c + cc) * 2 + (col & 1)] = acc;
  }
}

// ---- backward of the post-activation unit tail (bn_add_kernel): g = dy * [y > 0] (the ReLU after the
// residual add) written once, and in the same pass the backward reductions of the BatchNorm(s) that
// feed the add (sum g, sum g*(x - mean); rn_bn_bwd_part finalizes and applies them): the gradient
// and the BN inputs are not read a second time by separate reduction passes.
template <typename T, bool BNB, int NT = 0>
__global__ __launch_bounds__(256) void relu_bwd_bnred_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                             T* __restrict__ g, const T* __restrict__ xa,
                                                             const float* __restrict__ mean_a, float* __restrict__ part_a,
                                                             const T* __restrict__ xb,
                                                             const float* __restrict__ mean_b, float* __restrict__ part_b,
                                                             int64_t m, int c, int ct, int64_t rows_per_block) {
  constexpr int CE = 16 / sizeof(T);
  constexpr int NB = BNB ? 2 : 1;
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cbase = (blockIdx.x * ct + tc) * CE;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float mu[NB][CE], s[NB][CE], q[NB][CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    mu[0][e] = mean_a[cbase + e];
    if constexpr (BNB) mu[NB - 1][e] = mean_b[cbase + e];
#pragma unroll
    for (int b = 0; b < NB; ++b) s[b][e] = q[b][e] = 0.f;
  }
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    const int64_t off = r * c + cbase;
    float fy[CE], fd[CE], fx[NB][CE];
    chunk_to_f(ld16<NT>(y + off), fy, (const T*)nullptr);
    chunk_to_f(ld16<NT>(dy + off), fd, (const T*)nullptr);
    chunk_to_f(ld16<NT>(xa + off), fx[0], (const T*)nullptr);
    if constexpr (BNB) chunk_to_f(ld16<NT>(xb + off), fx[NB - 1], (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      fd[e] = fy[e] > 0.f ? fd[e] : 0.f;  // (exact in the storage type: dy or 0)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        s[b][e] += fd[e];
        q[b][e] = fmaf(fd[e], fx[b][e] - mu[b][e], q[b][e]);
      }
    }
    *reinterpret_cast<uint4*>(g + off) = f_to_chunk(fd, (const T*)nullptr);
  }
  __shared__ float red[kThreads * (8 * 2 + 1)];  // odd row stride: conflict-free LDS writes
  const int ncol = ct * CE * 2;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b > 0) __syncthreads();
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      red[(tr * ct + tc) * (CE * 2 + 1) + 2 * e] = s[b][e];
      red[(tr * ct + tc) * (CE * 2 + 1) + 2 * e + 1] = q[b][e];
    }
    __syncthreads();
    float* part = b == 0 ? part_a : part_b;
    for (int col = threadIdx.x; col < ncol; col += blockDim.x) {
      float acc = 0.f;
      const int tcv = col / (CE * 2), v = col - tcv * (CE * 2);
    for (int r = 0; r < rl; ++r) acc += red[(r * ct + tcv) * (CE * 2 + 1) + v];
      const int cc = blockIdx.x * ct * CE + col / 2;
      part[((int64_t)blockIdx.y * c + cc) * 2 + (col & 1)] = acc;
    }
  }
}

// coef[c] = {A = g*invstd, mean(dz), A2 = g*invstd^2*sum(dz*xhat)/m, mean}; block per channel.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nrb, int64_t m,
                                                              int c, int c_real, int fix_gamma,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ save_mean,
                                                              const float* __restrict__ save_invstd, float* dgamma,
                                                              float* dbeta, float* __restrict__ coef,
                                                              const float* __restrict__ global_var = nullptr,
                                                              float global_eps = 0.f) {
  const int ch = blockIdx.x;
  double s = 0.0, q = 0.0;
  for (int b0 = threadIdx.x; b0 < nrb; b0 += 8 * blockDim.x) {  // 8 loads in flight, summed in order
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = reinterpret_cast<const float2*>(part)[(int64_t)min(b0 + u * (int)blockDim.x, nrb - 1) * c + ch];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (b0 + u * (int)blockDim.x >= nrb) break;
      s += v[u].x;
      q += v[u].y;
    }
  }
  block_sum2(s, q);
  if (threadIdx.x != 0) return;
  if (ch >= c_real) {
    coef[ch * 4 + 0] = 0.f;
    coef[ch * 4 + 1] = 0.f;
    coef[ch * 4 + 2] = 0.f;
    coef[ch * 4 + 3] = 0.f;
    return;
  }
  // global statistics (use_global_stats, fix_bn: core/graph_optimize.py:114-157): save_invstd is
  // null, the normalisation used the moving statistics (save_mean = moving mean, invstd from the
  // moving variance and global_eps) and they are constants of the graph: dx = g*invstd*dz
  const bool global = save_invstd == nullptr;
  const double invstd = global ? 1.0 / sqrt((double)global_var[ch] + (double)global_eps) : (double)save_invstd[ch];
  const double g = fix_gamma ? 1.0 : (double)gamma[ch];
  const double dg_raw = q * invstd;  // sum dz * xhat
  if (dbeta) dbeta[ch] = (float)s;
  if (dgamma) dgamma[ch] = fix_gamma ? 0.f : (float)dg_raw;
  coef[ch * 4 + 0] = (float)(g * invstd);
  coef[ch * 4 + 1] = global ? 0.f : (float)(s / (double)m);
  coef[ch * 4 + 2] = global ? 0.f : (float)(g * invstd * invstd * dg_raw / (double)m);
  coef[ch * 4 + 3] = save_mean[ch];
}

template <typename T, bool RELU, bool PAIR = false, int NT = 0>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                           T* __restrict__ dx, const T* __restrict__ add,
                                                           const float* __restrict__ coef,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int64_t m, int c, int ct,
                                                           int64_t rows_per_block,
                                                           const float* __restrict__ clip = nullptr,
                                                           const T* __restrict__ dy2 = nullptr,
                                                           const float* __restrict__ clip2 = nullptr) {
  constexpr int CE = 16 / sizeof(T);
  const bool hc = clip != nullptr;
  const float t = hc ? *clip : 0.f;
  const float t2 = PAIR ? *clip2 : 0.f;
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cbase = (blockIdx.x * ct + tc) * CE;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float A[CE], mdz[CE], A2[CE], mu[CE], sc[CE], sh[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const float4 cf = reinterpret_cast<const float4*>(coef)[cbase + e];
    A[e] = cf.x;
    mdz[e] = cf.y;
    A2[e] = cf.z;
    mu[e] = cf.w;
    sc[e] = scale[cbase + e];
    sh[e] = shift[cbase + e];
  }
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    const int64_t off = r * c + cbase;
    float fx[CE], fd[CE], fa[CE], f2[CE];
    chunk_to_f(ld16<NT>(x + off), fx, (const T*)nullptr);
    chunk_to_f(ld16<NT>(dy + off), fd, (const T*)nullptr);
    if constexpr (PAIR) chunk_to_f(ld16<NT>(dy2 + off), f2, (const T*)nullptr);
    if (add) chunk_to_f(ld16<NT>(add + off), fa, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const float dz = PAIR ? relu_clip2_dz<T>(fx[e], sc[e], sh[e], fd[e], t, f2[e], t2)
                            : RELU ? fd[e] * relu_clip_mask<T>(fx[e], sc[e], sh[e], hc, t) : fd[e];
      float v = A[e] * (dz - mdz[e]) - A2[e] * (fx[e] - mu[e]);
      if (add) v += fa[e];
      fd[e] = v;
    }
    st16<NT>(dx + off, f_to_chunk(fd, (const T*)nullptr));
  }
}

// Elementwise (apply) geometry: same channel tiling as the reductions, more row blocks so
// that ~8 blocks per CU stream with every thread touching >= 8 rows.
template <typename T>
Geo make_apply_geo(int64_t m, int c) {
  Geo g = make_geo<T>(m, c);
  int64_t want = std::max<int64_t>(1, 4096 / g.gx);
  int64_t maxrb = std::max<int64_t>(1, m / (g.rl * 8));
  g.nrb = (int)std::min(want, maxrb);
  g.rows_per_block = ceil_div(m, g.nrb);
  return g;
}

template <typename T, bool RELU>
void launch_apply(const rn_bn_desc* d, const void* x, void* y, const float* scale, const float* shift,
                  hipStream_t st) {
  Geo a = make_apply_geo<T>(d->m, d->c);
  const int nt = (g_tune[RN_TUNE_BN_NT] & 32) ? 4 | (g_tune[RN_TUNE_BN_NT] & 2) : g_tune[RN_TUNE_BN_NT] & 3;
#define RN_APPLY(NT)                                                                                       \
  hipLaunchKernelGGL((bn_apply_kernel<T, RELU, NT>), dim3(a.gx, a.nrb), dim3(kThreads), 0, st, (const T*)x, \
                     (T*)y, scale, shift, d->m, d->c, a.ct, a.rows_per_block)
  if (nt == 1) RN_APPLY(1);
  else if (nt == 2) RN_APPLY(2);
  else if (nt == 3) RN_APPLY(3);
  else if (nt == 4) RN_APPLY(4);
  else if (nt == 6) RN_APPLY(6);
  else RN_APPLY(0);
#undef RN_APPLY
}

template <typename T, bool RELU>
void launch_bwd_apply(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add,
                      const float* coef, const float* scale, const float* shift, hipStream_t st) {
  Geo a = make_apply_geo<T>(d->m, d->c);
  const int nt = (g_tune[RN_TUNE_BN_NT] & 32) ? 4 | (g_tune[RN_TUNE_BN_NT] & 2) : g_tune[RN_TUNE_BN_NT] & 3;
  if (RELU && d->dy2)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true, true>), dim3(a.gx, a.nrb), dim3(kThreads), 0, st, (const T*)x,
                       (const T*)dy, (T*)dx, (const T*)add, coef, scale, shift, d->m, d->c, a.ct, a.rows_per_block,
                       d->clip, (const T*)d->dy2, d->clip2);
  else {
#define RN_BWD_APPLY(NT)                                                                                       \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RELU, false, NT>), dim3(a.gx, a.nrb), dim3(kThreads), 0, st,      \
                     (const T*)x, (const T*)dy, (T*)dx, (const T*)add, coef, scale, shift, d->m, d->c, a.ct,   \
                     a.rows_per_block, d->clip)
    if (nt == 1) RN_BWD_APPLY(1);
    else if (nt == 2) RN_BWD_APPLY(2);
    else if (nt == 3) RN_BWD_APPLY(3);
    else if (nt == 4) RN_BWD_APPLY(4);
    else if (nt == 6) RN_BWD_APPLY(6);
    else RN_BWD_APPLY(0);
#undef RN_BWD_APPLY
  }
}

template <typename T>
int bn_fwd_train_t(const rn_bn_desc* d, const void* x, void* y, const float* gamma, const float* beta,
                   float* mm, float* mv, float* smean, float* sinv, float* scale, float* shift, void* ws,
                   hipStream_t st) {
  Geo g = make_geo<T>(d->m, d->c);
  float* part = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(g.gx, g.nrb), dim3(kThreads), 0, st, (const T*)x, d->m,
                     d->c, g.ct, g.rows_per_block, part);
  hipLaunchKernelGGL(bn_fwd_finalize_kernel<T>, dim3(d->c), dim3(256), 0, st, (const T*)x, part,
                     g.nrb, d->m, d->c, d->c_real, d->eps, d->momentum, d->fix_gamma, gamma, beta, mm, mv,
                     smean, sinv, scale, shift);
  if (y) {
    if (d->relu) launch_apply<T, true>(d, x, y, scale, shift, st);
    else launch_apply<T, false>(d, x, y, scale, shift, st);
  }
  return rn_check_launch("bn_fwd_train");
}

template <typename T>
int bn_apply_t(const rn_bn_desc* d, const void* x, void* y, const float* scale, const float* shift,
               hipStream_t st) {
  if (d->relu) launch_apply<T, true>(d, x, y, scale, shift, st);
  else launch_apply<T, false>(d, x, y, scale, shift, st);
  return rn_check_launch("bn_apply");
}

template <typename T>
int bn_bwd_t(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add, const float* gamma,
             const float* smean, const float* sinv, const float* scale, const float* shift, float* dgamma,
             float* dbeta, void* ws, hipStream_t st, const float* global_var = nullptr) {
  Geo g = make_geo<T>(d->m, d->c);
  float* part = reinterpret_cast<float*>(ws);
  float* coef = part + (int64_t)g.nrb * d->c * 2;
  coef = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(coef) + 15) & ~uintptr_t(15));
  if (d->relu && d->dy2)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true, true>), dim3(g.gx, g.nrb), dim3(kThreads), 0, st, (const T*)x,
                       (const T*)dy, d->m, d->c, g.ct, g.rows_per_block, smean, scale, shift, part, d->clip,
                       (const T*)d->dy2, d->clip2);
  else if (d->relu && nt_reads())
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true, false, 2>), dim3(g.gx, g.nrb), dim3(kThreads), 0, st,
                       (const T*)x, (const T*)dy, d->m, d->c, g.ct, g.rows_per_block, smean, scale, shift, part,
                       d->clip);
  else if (d->relu)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true>), dim3(g.gx, g.nrb), dim3(kThreads), 0, st, (const T*)x,
                       (const T*)dy, d->m, d->c, g.ct, g.rows_per_block, smean, scale, shift, part, d->clip);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false>), dim3(g.gx, g.nrb), dim3(kThreads), 0, st, (const T*)x,
                       (const T*)dy, d->m, d->c, g.ct, g.rows_per_block, smean, scale, shift, part);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(d->c), dim3(256), 0, st, part, g.nrb, d->m, d->c,
                     d->c_real, d->fix_gamma, gamma, smean, global_var ? nullptr : sinv, dgamma, dbeta, coef,
                     global_var, d->eps);
  if (dx) {
    if (d->relu) launch_bwd_apply<T, true>(d, x, dy, dx, add, coef, scale, shift, st);
    else launch_bwd_apply<T, false>(d, x, dy, dx, add, coef, scale, shift, st);
  }
  return rn_check_launch("bn_bwd");
}

}  // namespace

extern "C" {

int64_t rn_bn_workspace_bytes(const rn_bn_desc* d) {
  Geo g = d->dtype == RN_BF16 ? make_geo<bf16_t>(d->m, d->c) : make_geo<float>(d->m, d->c);
  const int64_t stats = ((int64_t)g.nrb * d->c * 2 + (int64_t)d->c * 4) * (int64_t)sizeof(float) + 64;
  const int64_t merge = ceil_div(ceil_div(d->m, 128), kPartGroup) * 4 * d->c * (int64_t)sizeof(double) + 64;
  return std::max(stats, merge);  // rn_bn_fwd_train_part: 128-row producer blocks
}

static int check_bn(const rn_bn_desc* d) {
  RN_CHECK_ARG(d != nullptr, "null desc");
  RN_CHECK_ARG(d->dtype == RN_BF16 || d->dtype == RN_F32, "bad dtype");
  RN_CHECK_ARG(d->m > 0 && d->c > 0 && d->c % 8 == 0, "bad shape (c must be a multiple of 8)");
  RN_CHECK_ARG(d->c_real > 0 && d->c_real <= d->c, "bad c_real");
  RN_CHECK_ARG(!d->dy2 || (d->relu && d->clip && d->clip2), "dy2 needs relu, clip and clip2");
  return 0;
}

int rn_bn_fwd_train(const rn_bn_desc* d, const void* x, void* y, const float* gamma, const float* beta,
                    float* moving_mean, float* moving_var, float* save_mean, float* save_invstd, float* scale,
                    float* shift, void* ws, rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(x && beta && save_mean && save_invstd && scale && shift && ws, "null argument");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  RN_CHECK_ARG((moving_mean == nullptr) == (moving_var == nullptr), "moving stats must both be set");
  hipStream_t st = as_stream(stream);
  if (d->dtype == RN_BF16)
    return bn_fwd_train_t<bf16_t>(d, x, y, gamma, beta, moving_mean, moving_var, save_mean, save_invstd, scale,
                                  shift, ws, st);
  return bn_fwd_train_t<float>(d, x, y, gamma, beta, moving_mean, moving_var, save_mean, save_invstd, scale,
                               shift, ws, st);
}

int rn_bn_fwd_train_part(const rn_bn_desc* d, const float* part, int64_t nblk, int32_t rows_blk, int32_t ld,
                         const void* x, void* y, const float* gamma, const float* beta, float* moving_mean,
                         float* moving_var, float* save_mean, float* save_invstd, float* scale, float* shift,
                         void* ws, rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(part && nblk > 0 && rows_blk > 0 && ld >= d->c, "bad partials");
  RN_CHECK_ARG((int64_t)nblk * rows_blk >= d->m, "partials do not cover the rows");
  RN_CHECK_ARG(beta && save_mean && save_invstd && scale && shift, "null argument");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  RN_CHECK_ARG((moving_mean == nullptr) == (moving_var == nullptr), "moving stats must both be set");
  RN_CHECK_ARG(ws != nullptr, "null workspace");
  hipStream_t st = as_stream(stream);
  const int ngrp = (int)ceil_div(nblk, kPartGroup);
  double* part2 = reinterpret_cast<double*>(ws);
  if (ngrp <= 4 && g_tune[RN_TUNE_BN_MERGE] != 1) {  // (rn_set_tuning 24 = 1: the two launches everywhere)
    hipLaunchKernelGGL(bn_fwd_merge_finalize_kernel, dim3((d->c + 15) / 16), dim3(256), 0, st, part, (int)nblk,
                       d->m, rows_blk, ld, d->c, d->c_real, d->eps, d->momentum, d->fix_gamma, gamma, beta,
                       moving_mean, moving_var, save_mean, save_invstd, scale, shift);
  } else {
    hipLaunchKernelGGL(bn_part_merge_kernel, dim3((d->c + 63) / 64, ngrp), dim3(256), 0, st, part, (int)nblk, d->m,
                       rows_blk, ld, d->c, part2);
    hipLaunchKernelGGL(bn_fwd_finalize_part_kernel, dim3((d->c + 63) / 64), dim3(256), 0, st, part2, ngrp, d->m,
                       d->c, d->c_real, d->eps, d->momentum, d->fix_gamma, gamma, beta, moving_mean, moving_var,
                       save_mean, save_invstd, scale, shift);
  }
  if (rn_check_launch("bn_fwd_finalize_part")) return -1;
  if (!y) return 0;
  RN_CHECK_ARG(x != nullptr, "null x");
  if (d->dtype == RN_BF16) return bn_apply_t<bf16_t>(d, x, y, scale, shift, st);
  return bn_apply_t<float>(d, x, y, scale, shift, st);
}

namespace {
// the affine-transformed batch as the zero-bordered NHWC4 image: out[n][h + ph][w + pw][4] (bf16) of
// an image of hp x wp pixels whose border the caller zeroed once; thread per pixel, 8-byte stores
__global__ __launch_bounds__(256) void stem_to_nhwc4p_kernel(const float* __restrict__ x, int64_t npix, int c, int h,
                                                             int w, int hp, int wp, int ph, int pw,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, bf16_t* __restrict__ out) {
  const int hw = h * w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i / hw;
    const int pix = (int)(i - img * hw);
    const int hh = pix / w, ww = pix - hh * w;
    uint32_t packed[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float f = 0.f;
      if (e < c) {
        f = x[(img * c + e) * hw + pix];
        if (scale) f = fmaf(f, scale[e], shift[e]);
      }
      packed[e >> 1] |= (uint32_t)f2bf(f) << (16 * (e & 1));
    }
    const int64_t o = ((img * hp + hh + ph) * wp + ww + pw) * 4;
    *reinterpret_cast<uint2*>(out + o) = make_uint2(packed[0], packed[1]);
  }
}

int stem_prepare_impl(const rn_bn_desc* d, const float* x, int32_t n, int32_t c, int32_t h, int32_t w, void* out,
                      int32_t p4, int32_t hp, int32_t wp, int32_t ph, int32_t pw, int32_t mode, const float* gamma,
                      const float* beta, float* moving_mean, float* moving_var, float* save_mean, float* save_invstd,
                      float* scale, float* shift, void* ws, rn_stream_t stream);
}  // namespace

int rn_stem_prepare(const rn_bn_desc* d, const float* x, int32_t n, int32_t c, int32_t h, int32_t w, void* out,
                    int32_t mode, const float* gamma, const float* beta, float* moving_mean, float* moving_var,
                    float* save_mean, float* save_invstd, float* scale, float* shift, void* ws, rn_stream_t stream) {
  return stem_prepare_impl(d, x, n, c, h, w, out, 0, 0, 0, 0, 0, mode, gamma, beta, moving_mean, moving_var,
                           save_mean, save_invstd, scale, shift, ws, stream);
}

int rn_stem_prepare_p4(const rn_bn_desc* d, const float* x, int32_t n, int32_t c, int32_t h, int32_t w, void* out,
                       int32_t hp, int32_t wp, int32_t ph, int32_t pw, int32_t mode, const float* gamma,
                       const float* beta, float* moving_mean, float* moving_var, float* save_mean, float* save_invstd,
                       float* scale, float* shift, void* ws, rn_stream_t stream) {
  RN_CHECK_ARG(c <= 4 && ph >= 0 && pw >= 0 && hp >= h + ph && wp >= w + pw, "bad padded-image geometry");
  RN_CHECK_ARG(d && d->dtype == RN_BF16, "the padded NHWC4 image is bf16");
  return stem_prepare_impl(d, x, n, c, h, w, out, 1, hp, wp, ph, pw, mode, gamma, beta, moving_mean, moving_var,
                           save_mean, save_invstd, scale, shift, ws, stream);
}
}  // extern "C"

namespace {
int stem_prepare_impl(const rn_bn_desc* d, const float* x, int32_t n, int32_t c, int32_t h, int32_t w, void* out,
                      int32_t p4, int32_t hp, int32_t wp, int32_t ph, int32_t pw, int32_t mode, const float* gamma,
                      const float* beta, float* moving_mean, float* moving_var, float* save_mean, float* save_invstd,
                      float* scale, float* shift, void* ws, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && out && c >= 1 && c <= 8 && n > 0 && h > 0 && w > 0, "bad arguments");
  RN_CHECK_ARG(d->c == 8 && d->c_real == c && d->m == (int64_t)n * h * w, "desc must describe the NHWC-8 copy");
  RN_CHECK_ARG(mode == 2 || (beta && scale && shift), "affine outputs required");
  const int hw = h * w;
  RN_CHECK_ARG(hw % 4 == 0, "h*w must be a multiple of 4");
  hipStream_t st = as_stream(stream);
  if (mode == 0) {
    RN_CHECK_ARG(ws && save_mean && save_invstd && (d->fix_gamma || gamma), "null argument");
    const int nb = std::min(n, 256);
    const int ipb = (n + nb - 1) / nb;
    const int nbe = (n + ipb - 1) / ipb;
    float* part = reinterpret_cast<float*>(ws);
    hipLaunchKernelGGL(stem_stats_kernel, dim3(c, nbe), dim3(256), 0, st, x, n, c, hw, ipb, part);
    hipLaunchKernelGGL(stem_finalize_kernel, dim3(c), dim3(256), 0, st, x, part, nbe, d->m, c, hw, d->eps, d->momentum,
                       d->fix_gamma, gamma, beta, moving_mean, moving_var, save_mean, save_invstd, scale, shift);
  } else if (mode == 1) {
    RN_CHECK_ARG(moving_mean && moving_var && (d->fix_gamma || gamma), "null argument");
    hipLaunchKernelGGL(bn_infer_coef_kernel, dim3(1), dim3(64), 0, st, c, c, d->eps, d->fix_gamma, gamma, beta,
                       moving_mean, moving_var, scale, shift);
  }
  const float* sc = mode == 2 ? nullptr : scale;
  const float* sh = mode == 2 ? nullptr : shift;
  const int64_t npix = (int64_t)n * hw;
  const int grid = (int)std::min<int64_t>((npix + 255) / 256, 65536);
  if (p4) {
    hipLaunchKernelGGL(stem_to_nhwc4p_kernel, dim3(grid), dim3(256), 0, st, x, npix, c, h, w, hp, wp, ph, pw, sc, sh,
                       (bf16_t*)out);
    return rn_check_launch("stem_prepare_p4");
  }
  if (d->dtype == RN_BF16)
    hipLaunchKernelGGL(stem_to_nhwc8_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, x, npix, c, hw, sc, sh,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL(stem_to_nhwc8_kernel<float>, dim3(grid), dim3(256), 0, st, x, npix, c, hw, sc, sh,
                       (float*)out);
  return rn_check_launch("stem_prepare");
}
}  // namespace

extern "C" {

int rn_bn_bwd_part(const rn_bn_desc* d, const float* part, int64_t nrb, const void* x, const void* dy, void* dx,
                   const void* add_src, const float* gamma, const float* save_mean, const float* save_invstd,
                   const float* scale, const float* shift, float* dgamma, float* dbeta, void* ws,
                   rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(part && nrb > 0 && x && dy && save_mean && save_invstd && scale && shift && ws, "null argument");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  RN_CHECK_ARG(!d->dy2, "dy2: rn_bn_bwd only (the partials hold one gradient)");
  hipStream_t st = as_stream(stream);
  float* coef = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 15) & ~uintptr_t(15));
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(d->c), dim3(256), 0, st, part, (int)nrb, d->m, d->c, d->c_real,
                     d->fix_gamma, gamma, save_mean, save_invstd, dgamma, dbeta, coef);
  if (dx) {
    if (d->dtype == RN_BF16) {
      if (d->relu) launch_bwd_apply<bf16_t, true>(d, x, dy, dx, add_src, coef, scale, shift, st);
      else launch_bwd_apply<bf16_t, false>(d, x, dy, dx, add_src, coef, scale, shift, st);
    } else {
      if (d->relu) launch_bwd_apply<float, true>(d, x, dy, dx, add_src, coef, scale, shift, st);
      else launch_bwd_apply<float, false>(d, x, dy, dx, add_src, coef, scale, shift, st);
    }
  }
  return rn_check_launch("bn_bwd_part");
}


int rn_bn_bwd_finalize(const rn_bn_desc* d, const float* part, int64_t nrb, const float* gamma,
                       const float* save_mean, const float* save_invstd, float* dgamma, float* dbeta, float* coef,
                       rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(part && nrb > 0 && save_mean && save_invstd && coef, "null argument");
  RN_CHECK_ARG(((uintptr_t)coef & 15) == 0, "coef must be 16-byte aligned");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(d->c), dim3(256), 0, as_stream(stream), part, (int)nrb, d->m, d->c,
                     d->c_real, d->fix_gamma, gamma, save_mean, save_invstd, dgamma, dbeta, coef);
  return rn_check_launch("bn_bwd_finalize");
}

int rn_bn_fwd_infer(const rn_bn_desc* d, const void* x, void* y, const float* gamma, const float* beta,
                    const float* moving_mean, const float* moving_var, float* scale, float* shift,
                    rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(beta && moving_mean && moving_var && scale && shift, "null argument");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(bn_infer_coef_kernel, dim3((d->c + 255) / 256), dim3(256), 0, st, d->c, d->c_real, d->eps,
                     d->fix_gamma, gamma, beta, moving_mean, moving_var, scale, shift);
  if (!y) return rn_check_launch("bn_fwd_infer");  // coefficients only (consumer applies them)
  RN_CHECK_ARG(x != nullptr, "null x");
  if (d->dtype == RN_BF16) return bn_apply_t<bf16_t>(d, x, y, scale, shift, st);
  return bn_apply_t<float>(d, x, y, scale, shift, st);
}

int rn_bn_apply_add(const rn_bn_desc* d, const void* xa, const float* scale_a, const float* shift_a,
                    const void* xb, const float* scale_b, const float* shift_b, void* y, int32_t relu,
                    rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(xa && scale_a && shift_a && xb && y, "null argument");
  RN_CHECK_ARG((scale_b == nullptr) == (shift_b == nullptr), "scale_b / shift_b must both be set or both null");
  hipStream_t st = as_stream(stream);
  const bool bnb = scale_b != nullptr;
#define RN_BN_ADD(T, NT)                                                                                         \
  {                                                                                                            \
    Geo g = make_apply_geo<T>(d->m, d->c);                                                                     \
    dim3 gr(g.gx, g.nrb), bl(kThreads);                                                                        \
    if (relu && bnb) hipLaunchKernelGGL((bn_add_kernel<T, true, true, NT>), gr, bl, 0, st, (const T*)xa, scale_a,  \
                                        shift_a, (const T*)xb, scale_b, shift_b, (T*)y, d->m, d->c, g.ct,      \
                                        g.rows_per_block);                                                     \
    else if (relu) hipLaunchKernelGGL((bn_add_kernel<T, true, false, NT>), gr, bl, 0, st, (const T*)xa, scale_a,   \
                                      shift_a, (const T*)xb, scale_b, shift_b, (T*)y, d->m, d->c, g.ct,        \
                                      g.rows_per_block);                                                       \
    else if (bnb) hipLaunchKernelGGL((bn_add_kernel<T, false, true, NT>), gr, bl, 0, st, (const T*)xa, scale_a,    \
                                     shift_a, (const T*)xb, scale_b, shift_b, (T*)y, d->m, d->c, g.ct,         \
                                     g.rows_per_block);                                                        \
    else hipLaunchKernelGGL((bn_add_kernel<T, false, false, NT>), gr, bl, 0, st, (const T*)xa, scale_a, shift_a,   \
                            (const T*)xb, scale_b, shift_b, (T*)y, d->m, d->c, g.ct, g.rows_per_block);        \
  }
  if (d->dtype == RN_BF16 && nt_reads()) RN_BN_ADD(bf16_t, 2)
  else if (d->dtype == RN_BF16) RN_BN_ADD(bf16_t, 0)
  else RN_BN_ADD(float, 0)
#undef RN_BN_ADD
  return rn_check_launch("bn_apply_add");
}

int64_t rn_bn_reduce_blocks(const rn_bn_desc* d) {
  if (check_bn(d)) return -1;
  return d->dtype == RN_BF16 ? make_geo<bf16_t>(d->m, d->c).nrb : make_geo<float>(d->m, d->c).nrb;
}

int rn_relu_bwd_bnred(const rn_bn_desc* d, const void* y, const void* dy, void* g, const void* xa,
                      const float* mean_a, float* part_a, const void* xb, const float* mean_b, float* part_b,
                      rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(y && dy && g && xa && mean_a && part_a, "null argument");
  RN_CHECK_ARG((xb == nullptr) == (mean_b == nullptr) && (xb == nullptr) == (part_b == nullptr),
               "xb / mean_b / part_b must all be set or all null");
  hipStream_t st = as_stream(stream);
#define RN_RBR(T, NT)                                                                                           \
  {                                                                                                            \
    Geo gm = make_geo<T>(d->m, d->c);                                                                          \
    if (xb) hipLaunchKernelGGL((relu_bwd_bnred_kernel<T, true, NT>), dim3(gm.gx, gm.nrb), dim3(kThreads), 0, st,   \
                               (const T*)y, (const T*)dy, (T*)g, (const T*)xa, mean_a, part_a, (const T*)xb,   \
                               mean_b, part_b, d->m, d->c, gm.ct, gm.rows_per_block);                          \
    else hipLaunchKernelGGL((relu_bwd_bnred_kernel<T, false, NT>), dim3(gm.gx, gm.nrb), dim3(kThreads), 0, st,     \
                            (const T*)y, (const T*)dy, (T*)g, (const T*)xa, mean_a, part_a, (const T*)nullptr, \
                            (const float*)nullptr, (float*)nullptr, d->m, d->c, gm.ct, gm.rows_per_block);      \
  }
  if (d->dtype == RN_BF16 && nt_reads()) RN_RBR(bf16_t, 2)
  else if (d->dtype == RN_BF16) RN_RBR(bf16_t, 0)
  else RN_RBR(float, 0)
#undef RN_RBR
  return rn_check_launch("relu_bwd_bnred");
}

int rn_bn_apply(const rn_bn_desc* d, const void* x, void* y, const float* scale, const float* shift,
                rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(x && y && scale && shift, "null argument");
  hipStream_t st = as_stream(stream);
  if (d->dtype == RN_BF16) return bn_apply_t<bf16_t>(d, x, y, scale, shift, st);
  return bn_apply_t<float>(d, x, y, scale, shift, st);
}

int rn_bn_bwd(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add_src,
              const float* gamma, const float* save_mean, const float* save_invstd, const float* scale,
              const float* shift, float* dgamma, float* dbeta, void* ws, rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(x && dy && save_mean && save_invstd && scale && shift && ws, "null argument");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  hipStream_t st = as_stream(stream);
  if (d->dtype == RN_BF16)
    return bn_bwd_t<bf16_t>(d, x, dy, dx, add_src, gamma, save_mean, save_invstd, scale, shift, dgamma, dbeta,
                            ws, st);
  return bn_bwd_t<float>(d, x, dy, dx, add_src, gamma, save_mean, save_invstd, scale, shift, dgamma, dbeta, ws,
                         st);
}

int rn_bn_bwd_apply_rows(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add_src,
                         const float* scale, const float* shift, const void* ws, int64_t row0, int64_t rows,
                         rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(x && dy && dx && scale && shift && ws, "null argument");
  RN_CHECK_ARG(!d->dy2, "dy2: rn_bn_bwd only");
  RN_CHECK_ARG(row0 >= 0 && rows > 0 && row0 + rows <= d->m, "row range outside the tensor");
  const int64_t es = d->dtype == RN_BF16 ? 2 : 4;
  RN_CHECK_ARG(row0 * d->c * es % 16 == 0, "row0 * c must be a whole number of 16-byte chunks");
  // the coefficients rn_bn_bwd (dx = NULL) left in ws, located by the whole tensor's geometry
  Geo g = d->dtype == RN_BF16 ? make_geo<bf16_t>(d->m, d->c) : make_geo<float>(d->m, d->c);
  const float* coef = reinterpret_cast<const float*>(ws) + (int64_t)g.nrb * d->c * 2;
  coef = reinterpret_cast<const float*>((reinterpret_cast<uintptr_t>(coef) + 15) & ~uintptr_t(15));
  rn_bn_desc dd = *d;
  dd.m = rows;
  const int64_t off = row0 * d->c * es;
  auto at = [&](const void* p) { return p ? (const void*)((const char*)p + off) : nullptr; };
  hipStream_t st = as_stream(stream);
  void* dxo = (char*)dx + off;
  if (d->dtype == RN_BF16) {
    if (d->relu) launch_bwd_apply<bf16_t, true>(&dd, at(x), at(dy), dxo, at(add_src), coef, scale, shift, st);
    else launch_bwd_apply<bf16_t, false>(&dd, at(x), at(dy), dxo, at(add_src), coef, scale, shift, st);
  } else {
    if (d->relu) launch_bwd_apply<float, true>(&dd, at(x), at(dy), dxo, at(add_src), coef, scale, shift, st);
    else launch_bwd_apply<float, false>(&dd, at(x), at(dy), dxo, at(add_src), coef, scale, shift, st);
  }
  return rn_check_launch("bn_bwd_apply_rows");
}

int rn_bn_bwd_global(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add_src,
                     const float* gamma, const float* moving_mean, const float* moving_var, const float* scale,
                     const float* shift, float* dgamma, float* dbeta, void* ws, rn_stream_t stream) {
  if (check_bn(d)) return -1;
  RN_CHECK_ARG(x && dy && moving_mean && moving_var && scale && shift && ws, "null argument");
  RN_CHECK_ARG(d->fix_gamma || gamma, "gamma required unless fix_gamma");
  hipStream_t st = as_stream(stream);
  if (d->dtype == RN_BF16)
    return bn_bwd_t<bf16_t>(d, x, dy, dx, add_src, gamma, moving_mean, nullptr, scale, shift, dgamma, dbeta, ws,
                            st, moving_var);
  return bn_bwd_t<float>(d, x, dy, dx, add_src, gamma, moving_mean, nullptr, scale, shift, dgamma, dbeta, ws, st,
                         moving_var);
}

}  // extern "C"
