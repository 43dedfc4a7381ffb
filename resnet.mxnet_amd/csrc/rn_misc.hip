// rn_misc.hip -- pooling, SoftmaxOutput, SGD-momentum, int8 fake-quant, casts, runtime info.
//
// Pooling       : mx.sym.Pooling (reference symbol/resnet.py:97 max 3x3/s2/p1, :113 global avg)
// SoftmaxOutput : mx.sym.SoftmaxOutput (symbol/resnet.py:118-120), grad = p - onehot, 'null' norm
// SGD momentum  : optimizer 'sgd' with momentum/wd/rescale_grad (train.py:186-194)
// Quantization  : mx.sym.contrib.Quantization_int8 (symbol/int8_api.py:133-136) with the
//                 semantics of symbol/quant_ops.py:12-42 and clip_grad_quantization_int8.py:14-67
#include <algorithm>
#include <cstring>

#include "rn_common.h"

static thread_local std::string g_last_error;
void rn_set_error(const std::string& msg) { g_last_error = msg; }
int rn_check_launch(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    rn_set_error(std::string(where) + ": " + hipGetErrorString(e));
    return -1;
  }
  return 0;
}

namespace {

int grid1d(int64_t total, int block = 256, int cap = 8192) {
  int64_t g = (total + block - 1) / block;
  return (int)std::min<int64_t>(std::max<int64_t>(g, 1), cap);
}

// ------------------------------------------------------------------------------ pooling
struct PoolArgs {
  int n, h, w, c, r, s, sh, sw, ph, pw, p, q, type;
  FastDiv fd_cpr, fd_a, fd_b;  // chunks per pixel; fwd: q, p / bwd: w, h (32-bit index math)
};

// forward: thread per (output pixel, chunk). Max: first maximal tap in (r, s) scan order,
// which is the element MXNet's max-unpool gives the gradient to. Avg: count_include_pad
// (divisor r*s), global pool divides by h*w. XF: x is the input of the producing BatchNorm+ReLU, applied
// per loaded element and rounded to T exactly as bn_apply_kernel stores it (max(x sc + sh, 0)), so the
// pooled values and tap indices are bit-identical to pooling the stored activation, which is never written.
template <typename T, bool XF = false>
__global__ void pool_fwd_kernel(PoolArgs a, const T* __restrict__ x, T* __restrict__ y,
                                uint8_t* __restrict__ argmax, const float* __restrict__ in_sc = nullptr,
                                const float* __restrict__ in_sh = nullptr) {
  constexpr int CE = 16 / sizeof(T);
  const int cpr = a.c / CE;
  const uint32_t total = (uint32_t)a.n * a.p * a.q * cpr;  // host-checked < 2^31
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = fdiv(i, a.fd_cpr);
    const int cc = (int)(i - pix * cpr);
    const uint32_t t = fdiv(pix, a.fd_a);
    const int qq = (int)(pix - t * a.q);
    const uint32_t n = fdiv(t, a.fd_b);
    const int pp = (int)(t - n * a.p);
    float xs[CE], xh[CE];
    if constexpr (XF)
#pragma unroll
      for (int e = 0; e < CE; ++e) {
        xs[e] = in_sc[cc * CE + e];
        xh[e] = in_sh[cc * CE + e];
      }
    auto act = [&](float (&f)[CE]) __attribute__((always_inline)) {
      if constexpr (XF)
#pragma unroll
        for (int e = 0; e < CE; ++e) f[e] = to_f(from_f<T>(fmaxf(fmaf(f[e], xs[e], xh[e]), 0.f)));
    };
    float best[CE];
    int arg[CE];
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      best[e] = a.type == RN_POOL_MAX ? -INFINITY : 0.f;
      arg[e] = 0;
    }
    if (a.type == RN_POOL_MAX && a.r == 3 && a.s == 3) {
      // the ResNet stem pool: all 9 window loads issued before the first max (clamped addresses,
      // out-of-image taps masked), so they are in flight together
      uint4 v[9];
      bool ok[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int hh = pp * a.sh - a.ph + r, ww = qq * a.sw - a.pw + s;
          ok[r * 3 + s] = (unsigned)hh < (unsigned)a.h && (unsigned)ww < (unsigned)a.w;
          const int hc = ok[r * 3 + s] ? hh : 0, wc = ok[r * 3 + s] ? ww : 0;
          v[r * 3 + s] = *reinterpret_cast<const uint4*>(x + (((int64_t)n * a.h + hc) * a.w + wc) * a.c + cc * CE);
        }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        float f[CE];
        chunk_to_f(v[t], f, (const T*)nullptr);
        act(f);
#pragma unroll
        for (int e = 0; e < CE; ++e)
          if (ok[t] && f[e] > best[e]) {
            best[e] = f[e];
            arg[e] = t;
          }
      }
    } else
    for (int r = 0; r < a.r; ++r) {
      const int hh = pp * a.sh - a.ph + r;
      if (hh < 0 || hh >= a.h) continue;
      for (int s = 0; s < a.s; ++s) {
        const int ww = qq * a.sw - a.pw + s;
        if (ww < 0 || ww >= a.w) continue;
        float f[CE];
        chunk_to_f(*reinterpret_cast<const uint4*>(x + (((int64_t)n * a.h + hh) * a.w + ww) * a.c + cc * CE), f,
                   (const T*)nullptr);
        act(f);
#pragma unroll
        for (int e = 0; e < CE; ++e) {
          if (a.type == RN_POOL_MAX) {
            if (f[e] > best[e]) {
              best[e] = f[e];
              arg[e] = r * a.s + s;
            }
          } else {
            best[e] += f[e];
          }
        }
      }
    }
    if (a.type != RN_POOL_MAX) {
      const float inv = 1.f / (float)(a.r * a.s);
#pragma unroll
      for (int e = 0; e < CE; ++e) best[e] *= inv;
    } else if (argmax) {  // the chunk's CE tap indices in one 8- or 4-byte store
      uint64_t packed = 0;
#pragma unroll
      for (int e = 0; e < CE; ++e) packed |= (uint64_t)(uint8_t)arg[e] << (8 * e);
      if (CE == 8) *reinterpret_cast<uint64_t*>(argmax + pix * a.c + cc * CE) = packed;
      else *reinterpret_cast<uint32_t*>(argmax + pix * a.c + cc * CE) = (uint32_t)packed;
    }
    reinterpret_cast<uint4*>(y)[i] = f_to_chunk(best, (const T*)nullptr);
  }
}

// backward: input-centric gather (deterministic, no atomics).
template <typename T>
__global__ void pool_bwd_kernel(PoolArgs a, const T* __restrict__ dy, const uint8_t* __restrict__ argmax,
                                T* __restrict__ dx, const T* __restrict__ add) {
  constexpr int CE = 16 / sizeof(T);
  const int cpr = a.c / CE;
  const uint32_t total = (uint32_t)a.n * a.h * a.w * cpr;  // host-checked < 2^31
  const float inv = 1.f / (float)(a.r * a.s);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = fdiv(i, a.fd_cpr);
    const int cc = (int)(i - pix * cpr);
    const uint32_t t = fdiv(pix, a.fd_a);
    const int ww = (int)(pix - t * a.w);
    const uint32_t n = fdiv(t, a.fd_b);
    const int hh = (int)(t - n * a.h);
    float acc[CE];
    if (add) chunk_to_f(reinterpret_cast<const uint4*>(add)[i], acc, (const T*)nullptr);
    else
#pragma unroll
      for (int e = 0; e < CE; ++e) acc[e] = 0.f;
    // outputs whose window contains hh: pp*sh - ph <= hh <= pp*sh - ph + r - 1
    int plo = hh + a.ph - a.r + 1;
    plo = plo <= 0 ? 0 : (plo + a.sh - 1) / a.sh;
    const int phi = min(a.p - 1, (hh + a.ph) / a.sh);
    int qlo = ww + a.pw - a.s + 1;
    qlo = qlo <= 0 ? 0 : (qlo + a.sw - 1) / a.sw;
    const int qhi = min(a.q - 1, (ww + a.pw) / a.sw);
    if (a.type == RN_POOL_MAX && a.r == 3 && a.s == 3 && a.sh == 2 && a.sw == 2) {
      // 3x3 / stride 2: at most 2 x 2 windows hold this pixel; their dy chunks and tap indices are
      // loaded together (clamped addresses, masked), then added in the generic order
      uint4 g4[4];
      uint64_t am4[4];
      bool ok4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int pp = plo + (u >> 1), qq = qlo + (u & 1);
        ok4[u] = pp <= phi && qq <= qhi;
        const int64_t obase = (((int64_t)n * a.p + (ok4[u] ? pp : 0)) * a.q + (ok4[u] ? qq : 0)) * a.c + cc * CE;
        g4[u] = *reinterpret_cast<const uint4*>(dy + obase);
        am4[u] = CE == 8 ? *reinterpret_cast<const uint64_t*>(argmax + obase)
                         : (uint64_t)*reinterpret_cast<const uint32_t*>(argmax + obase);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int pp = plo + (u >> 1), qq = qlo + (u & 1);
        const int tap = (hh - (pp * 2 - a.ph)) * 3 + (ww - (qq * 2 - a.pw));
        float g[CE];
        chunk_to_f(g4[u], g, (const T*)nullptr);
#pragma unroll
        for (int e = 0; e < CE; ++e)
          if (ok4[u] && (int)((am4[u] >> (8 * e)) & 0xFF) == tap) acc[e] += g[e];
      }
      reinterpret_cast<uint4*>(dx)[i] = f_to_chunk(acc, (const T*)nullptr);
      continue;
    }
    for (int pp = plo; pp <= phi; ++pp) {
      const int r = hh - (pp * a.sh - a.ph);
      for (int qq = qlo; qq <= qhi; ++qq) {
        const int s = ww - (qq * a.sw - a.pw);
        const int tap = r * a.s + s;
        const int64_t obase = (((int64_t)n * a.p + pp) * a.q + qq) * a.c + cc * CE;
        float g[CE];
        chunk_to_f(*reinterpret_cast<const uint4*>(dy + obase), g, (const T*)nullptr);
        if (a.type == RN_POOL_MAX) {  // the chunk's CE tap indices in one 8- or 4-byte load
          const uint64_t am = CE == 8 ? *reinterpret_cast<const uint64_t*>(argmax + obase)
                                      : (uint64_t)*reinterpret_cast<const uint32_t*>(argmax + obase);
#pragma unroll
          for (int e = 0; e < CE; ++e)
            if ((int)((am >> (8 * e)) & 0xFF) == tap) acc[e] += g[e];
        } else {
#pragma unroll
          for (int e = 0; e < CE; ++e) acc[e] += g[e] * inv;
        }
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = f_to_chunk(acc, (const T*)nullptr);
  }
}

// ------------------------------------------------------------------------------ softmax
// one wave per sample row
template <typename GT>
__global__ void softmax_output_kernel(int batch, int ncls, int ld, const float* __restrict__ logits,
                                      const float* __restrict__ label, float* __restrict__ prob,
                                      GT* __restrict__ dlogits, float grad_scale, float* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= batch) return;
  const float* z = logits + (int64_t)row * ld;
  float mx = -INFINITY;
  for (int j = lane; j < ncls; j += 64) mx = fmaxf(mx, z[j]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < ncls; j += 64) sum += __expf(z[j] - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  const int lab = (int)label[row];
  const float zl = (lab >= 0 && lab < ncls) ? z[lab] : -INFINITY;
  float greater = 0.f, equal_before = 0.f;
  for (int j = lane; j < ld; j += 64) {
    if (j < ncls) {
      const float pj = __expf(z[j] - mx) * inv;
      if (prob) prob[(int64_t)row * ncls + j] = pj;
      const float gj = grad_scale * (pj - (j == lab ? 1.f : 0.f));
      if (dlogits) dlogits[(int64_t)row * ld + j] = from_f<GT>(gj);
      greater += z[j] > zl ? 1.f : 0.f;
      equal_before += (z[j] == zl && j < lab) ? 1.f : 0.f;
    } else if (dlogits) {
      dlogits[(int64_t)row * ld + j] = from_f<GT>(0.f);
    }
  }
  greater = wave_sum(greater);
  equal_before = wave_sum(equal_before);
  if (lane == 0 && stats) {
    const float logp = zl - mx - __logf(sum);
    atomicAdd(stats + 0, -logp);
    atomicAdd(stats + 1, (greater == 0.f && equal_before == 0.f) ? 1.f : 0.f);
    atomicAdd(stats + 2, greater < 5.f ? 1.f : 0.f);
  }
}

template <typename T>
__global__ void col_sum_kernel(int64_t m, int c, int ld, const T* __restrict__ x, float* __restrict__ out,
                               int accumulate) {
  const int j = blockIdx.x;
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < m; i += blockDim.x) acc += to_f(x[i * ld + j]);
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = accumulate ? out[j] + red[0] : red[0];
}

// ------------------------------------------------------------------------------ SGD
template <typename LT>
__global__ void sgd_mom_kernel(const int64_t* __restrict__ offs, const int64_t* __restrict__ numels,
                               const float* __restrict__ wds, float* __restrict__ w, const float* __restrict__ g,
                               float* __restrict__ mom, LT* __restrict__ wl, float lr, const float* lr_dev,
                               float momentum, float rescale, float clip) {
  const int t = blockIdx.y;
  const int64_t off = offs[t], n = numels[t];
  const float wd = wds[t];
  const float lrv = lr_dev ? *lr_dev : lr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = off + i;
    float gr = rescale * g[k];
    if (clip > 0.f) gr = fminf(fmaxf(gr, -clip), clip);
    const float wv = w[k];
    const float mv = momentum * mom[k] - lrv * (gr + wd * wv);
    mom[k] = mv;
    const float nw = wv + mv;
    w[k] = nw;
    if (wl) wl[k] = from_f<LT>(nw);
  }
}

// SGD momentum with the compute copies written in the same pass. A conv/FC master tensor is KRSC
// over creal channels (index (k*RS + tap)*creal + ci); its copies are KRSC over the channel stride c
// and CRSK over the output stride kpad (the layouts pack_krsc/pack_crsk write). One workgroup per
// work item: a 4096-element chunk of a tensor without a CRSK copy, or a 64(k) x 64(ci) tile of one
// tap, transposed through LDS so both copies are written with coalesced rows.
// Padding entries of the copies are never touched (zero since the bind-time pack).
constexpr int kSgdChunk = 4096;
template <typename LT, bool CHECK = false>
__global__ __launch_bounds__(256) void sgd_mom_pack_kernel(const int64_t* __restrict__ offs,
                                                           const float* __restrict__ wds, float* __restrict__ w,
                                                           const float* __restrict__ g, float* __restrict__ mom,
                                                           const rn_wpack* __restrict__ packs,
                                                           const int4* __restrict__ work, const int64_t* numels,
                                                           float lr, const float* lr_dev, float momentum,
                                                           float rescale, float clip, const int64_t* lim = nullptr,
                                                           int* flag = nullptr) {
  __shared__ LT tile[64][65];
  const int4 wi = work[blockIdx.x];
  const int t = wi.x;
  const int64_t off = offs[t];
  const float wd = wds[t];
  const float lrv = lr_dev ? *lr_dev : lr;
  const rn_wpack pk = packs[t];
  LT* __restrict__ wk = reinterpret_cast<LT*>(pk.krsc);
  LT* __restrict__ wc = reinterpret_cast<LT*>(pk.crsk);
  auto upd = [&](int64_t k) __attribute__((always_inline)) {
    if (CHECK && (k < 0 || k >= lim[0])) {
      atomicOr(flag, 1);
      return 0.f;
    }
    float gr = rescale * g[k];
    if (clip > 0.f) gr = fminf(fmaxf(gr, -clip), clip);
    const float wv = w[k];
    const float mv = momentum * mom[k] - lrv * (gr + wd * wv);
    mom[k] = mv;
    const float nw = wv + mv;
    w[k] = nw;
    return nw;
  };
  if (!wc) {  // elementwise chunk [wi.y, wi.y + kSgdChunk)
    const int n = (int)min<int64_t>(numels[t], (int64_t)wi.y + kSgdChunk);
    for (int i = wi.y + threadIdx.x; i < n; i += 256) {
      const float nw = upd(off + i);
      if (wk) {
        const int64_t o = (int64_t)(i / pk.creal) * pk.c + i % pk.creal;
        if (CHECK && (o < 0 || o >= lim[1 + 2 * t])) {
          atomicOr(flag, 2);
          continue;
        }
        wk[o] = from_f<LT>(nw);
      }
    }
    return;
  }
  const int k0 = wi.y, tap = wi.z, c0 = wi.w;
  const int cl = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {  // rows k0 + r, columns c0 + cl: coalesced over ci
    const int r = r0 + 4 * j, k = k0 + r, ci = c0 + cl;
    if (k < pk.k && ci < pk.creal) {
      const int64_t kt = (int64_t)k * pk.rs + tap;
      const LT v = from_f<LT>(upd(off + kt * pk.creal + ci));
      if (CHECK && (kt * pk.c + ci >= lim[1 + 2 * t])) atomicOr(flag, 4);
      else wk[kt * pk.c + ci] = v;
      tile[r][cl] = v;
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {  // rows ci, columns k: coalesced over k
    const int r = r0 + 4 * j, ci = c0 + r, k = k0 + cl;
    if (k < pk.k && ci < pk.creal) {
      const int64_t o = ((int64_t)ci * pk.rs + tap) * pk.kpad + k;
      if (CHECK && o >= lim[2 + 2 * t]) atomicOr(flag, 8);
      else wc[o] = tile[cl][r];
    }
  }
}

// ------------------------------------------------------------------------------ layout / casts
template <typename T>
__global__ void nchw_to_nhwc_kernel(int n, int c, int h, int w, int cpad, const float* __restrict__ src,
                                    T* __restrict__ dst) {
  const int64_t total = (int64_t)n * h * w * cpad;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpad);
    const int64_t pix = i / cpad;
    const int ww = (int)(pix % w);
    const int hh = (int)((pix / w) % h);
    const int nn = (int)(pix / ((int64_t)w * h));
    const float v = cc < c ? src[(((int64_t)nn * c + cc) * h + hh) * w + ww] : 0.f;
    dst[i] = from_f<T>(v);
  }
}

template <typename S, typename D>
__global__ void cast_kernel(int64_t n, const S* __restrict__ src, D* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = from_f<D>(to_f(src[i]));
}

// 16-byte chunks; n must be a multiple of the chunk (activation buffers always are)
template <typename T, bool RELU>
__global__ void add_kernel(int64_t nchunk, const T* a, const T* b, T* dst) {
  constexpr int CE = 16 / sizeof(T);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunk; i += (int64_t)gridDim.x * blockDim.x) {
    float fa[CE], fb[CE];
    chunk_to_f(reinterpret_cast<const uint4*>(a)[i], fa, (const T*)nullptr);
    if (b) chunk_to_f(reinterpret_cast<const uint4*>(b)[i], fb, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      float v = b ? fa[e] + fb[e] : fa[e];
      fa[e] = RELU ? fmaxf(v, 0.f) : v;
    }
    reinterpret_cast<uint4*>(dst)[i] = f_to_chunk(fa, (const T*)nullptr);
  }
}
template <typename T>
__global__ void relu_bwd_kernel(int64_t nchunk, const T* __restrict__ y, const T* __restrict__ dy, T* __restrict__ dx,
                                const T* __restrict__ add) {
  constexpr int CE = 16 / sizeof(T);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunk; i += (int64_t)gridDim.x * blockDim.x) {
    float fy[CE], fd[CE], fa[CE];
    chunk_to_f(reinterpret_cast<const uint4*>(y)[i], fy, (const T*)nullptr);
    chunk_to_f(reinterpret_cast<const uint4*>(dy)[i], fd, (const T*)nullptr);
    if (add) chunk_to_f(reinterpret_cast<const uint4*>(add)[i], fa, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      float v = fy[e] > 0.f ? fd[e] : 0.f;
      fd[e] = add ? v + fa[e] : v;
    }
    reinterpret_cast<uint4*>(dx)[i] = f_to_chunk(fd, (const T*)nullptr);
  }
}

// ------------------------------------------------------------------------------ int8 quant
template <typename T>
__global__ void absmax_kernel(int64_t n, const T* __restrict__ x, float* __restrict__ out) {
  // 16-byte chunks (x is 16-byte aligned: device allocations / tensor offsets), then the tail
  constexpr int CE = 16 / sizeof(T);
  const int64_t nc = n / CE;
  float m = 0.f;
#pragma unroll 4
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nc; i += (int64_t)gridDim.x * blockDim.x) {
    float f[CE];
    chunk_to_f(reinterpret_cast<const uint4*>(x)[i], f, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) m = fmaxf(m, fabsf(f[e]));
  }
  for (int64_t i = nc * CE + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(to_f(x[i])));
  m = wave_max(m);
  // one atomic per block (thousands of same-address atomics serialise in L2)
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  // non-negative floats order like their bit patterns
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}
// curmax is consumed and re-zeroed here (the next quantizer sharing the workspace starts from 0: no
// memset launch per call); unit (nullable) = t / qmax for the int8 codes' consumers
__global__ void quant_state_kernel(float* __restrict__ curmax, float* minmax, int is_weight, int is_train,
                                   float decay, int first, float* __restrict__ thr, float qmax = 1.f,
                                   float* __restrict__ unit = nullptr) {
  const float t = quant_state_update(*curmax, minmax, is_weight, is_train, decay, first);
  *thr = t;
  *curmax = 0.f;
  if (unit) *unit = t / qmax;
}
template <typename T>
__global__ void quant_apply_kernel(int64_t n, const T* __restrict__ x, T* __restrict__ out,
                                   const float* __restrict__ thr, float qmax, int clip) {
  const float t = *thr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = from_f<T>(quant_value(to_f(x[i]), t, qmax, clip));
}
// fake-quantized values AND their int8 codes, 16 elements (one 16-byte code chunk) per thread:
// code = round(clip(v) / unit) (the value quant_value returns is code * unit), unit[0] = t / qmax
template <typename T>
__global__ void quant_codes_kernel(int64_t nchunk, const T* __restrict__ x, T* __restrict__ out,
                                   int8_t* __restrict__ codes, const float* __restrict__ thr, float qmax, int clip,
                                   float* __restrict__ unit_out) {
  const float t = *thr;
  const float unit = t / qmax;
  if (blockIdx.x == 0 && threadIdx.x == 0 && unit_out) *unit_out = unit;
  constexpr int CE = 16 / sizeof(T);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunk; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t cw[4];
#pragma unroll
    for (int h = 0; h < 16 / CE; ++h) {
      float f[CE];
      chunk_to_f(reinterpret_cast<const uint4*>(x)[i * (16 / CE) + h], f, (const T*)nullptr);
#pragma unroll
      for (int e = 0; e < CE; ++e) {
        float v = clip ? fminf(fmaxf(f[e], -t), t) : f[e];
        const float q = unit > 0.f ? roundf(v / unit) : 0.f;
        f[e] = q * unit;
        const int j = h * CE + e;
        const uint32_t b = (uint32_t)(uint8_t)(int8_t)(int)q;
        if ((j & 3) == 0) cw[j >> 2] = b;
        else cw[j >> 2] |= b << (8 * (j & 3));
      }
      if (out) reinterpret_cast<uint4*>(out)[i * (16 / CE) + h] = f_to_chunk(f, (const T*)nullptr);
    }
    reinterpret_cast<uint4*>(codes)[i] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
  }
}
// the fake-quantized values from the codes: out = code * unit rounded to T -- the same fp32 product
// the quantizer kernels round (bit-identical to their out), 16 elements per thread
template <typename T>
__global__ void quant_expand_kernel(int64_t nchunk, const int8_t* __restrict__ codes, const float* __restrict__ unit_p,
                                    T* __restrict__ out) {
  const float unit = *unit_p;
  constexpr int CE = 16 / sizeof(T);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunk; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 cw = reinterpret_cast<const uint4*>(codes)[i];
    const uint32_t w[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
    for (int h = 0; h < 16 / CE; ++h) {
      float f[CE];
#pragma unroll
      for (int e = 0; e < CE; ++e) {
        const int j = h * CE + e;
        f[e] = (float)(int8_t)((w[j >> 2] >> (8 * (j & 3))) & 0xFF) * unit;
      }
      reinterpret_cast<uint4*>(out)[i * (16 / CE) + h] = f_to_chunk(f, (const T*)nullptr);
    }
  }
}
template <typename T>
__global__ void quant_bwd_kernel(int64_t n, const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx,
                                 const float* __restrict__ minmax, int is_weight, const T* __restrict__ add) {
  const float t = (is_weight || !minmax) ? INFINITY : *minmax;
  constexpr int CE = 16 / sizeof(T);
  const int64_t nc = n / CE;  // 16-byte chunks, then the tail
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nc; i += (int64_t)gridDim.x * blockDim.x) {
    float fx[CE], fd[CE], fa[CE];
    chunk_to_f(reinterpret_cast<const uint4*>(x)[i], fx, (const T*)nullptr);
    chunk_to_f(reinterpret_cast<const uint4*>(dy)[i], fd, (const T*)nullptr);
    if (add) chunk_to_f(reinterpret_cast<const uint4*>(add)[i], fa, (const T*)nullptr);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      float g = fd[e];
      if (!is_weight && !(fx[e] > -t && fx[e] < t)) g = 0.f;
      fd[e] = add ? g + fa[e] : g;
    }
    reinterpret_cast<uint4*>(dx)[i] = f_to_chunk(fd, (const T*)nullptr);
  }
  for (int64_t i = nc * CE + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xv = to_f(x[i]);
    float g = to_f(dy[i]);
    if (!is_weight && !(xv > -t && xv < t)) g = 0.f;
    if (add) g += to_f(add[i]);
    dx[i] = from_f<T>(g);
  }
}

// ---- Quantization_int8 of a BatchNorm(+ReLU) output, the BatchNorm applied on load
// (rn_quant_int8_fwd_codes_bn). Thread = one 16-channel group (one 16-byte code chunk) of the rows
// r0 + tr, r0 + tr + rl, ...; y = [relu](fmaf(x, scale, shift)) rounded to T exactly as bn_apply_kernel
// stores it, so max|y|, the codes and the fake-quantized values equal rn_bn_apply followed by
// rn_quant_int8_fwd_codes bit for bit, without the BatchNorm output's write and two re-reads.
typedef unsigned int bnq_u32x4 __attribute__((ext_vector_type(4)));
template <typename T, bool RELU, bool NT = false>
__device__ __forceinline__ void bnq_load(const T* __restrict__ x, const float* sc, const float* sh, float* f) {
  constexpr int CE = 16 / sizeof(T);
#pragma unroll
  for (int h = 0; h < 16 / CE; ++h) {
    uint4 u;
    if constexpr (NT) {  // rn_set_tuning 18 bit 8: the streaming hint (as rn_bn.hip's BatchNorm passes)
      const bnq_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const bnq_u32x4*>(x) + h);
      u = make_uint4(v.x, v.y, v.z, v.w);
    } else {
      u = reinterpret_cast<const uint4*>(x)[h];
    }
    chunk_to_f(u, f + h * CE, (const T*)nullptr);
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float v = fmaf(f[e], sc[e], sh[e]);
    f[e] = to_f(from_f<T>(RELU ? fmaxf(v, 0.f) : v));
  }
}
template <typename T, bool RELU>
__global__ __launch_bounds__(256) void bnq_absmax_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int64_t m, int c, int ct,
                                                         int64_t rows_per_block, float* __restrict__ out) {
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  const int cb = (blockIdx.x * ct + tc) * 16;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  float mx = 0.f;
  if (tr < rl) {  // (256 % ct threads idle)
    float sc[16], sh[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      sc[e] = scale[cb + e];
      sh[e] = shift[cb + e];
    }
    for (int64_t r = r0 + tr; r < r1; r += rl) {
      float f[16];
      bnq_load<T, RELU>(x + r * c + cb, sc, sh, f);
#pragma unroll
      for (int e = 0; e < 16; ++e) mx = fmaxf(mx, fabsf(f[e]));
    }
  }
  mx = wave_max(mx);
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}
// max y of y = relu(x*scale + shift) (rounded to T) from the per-block per-channel extremes of x
// (rn_bn_desc.xmm: the max where scale >= 0, else the min): y is monotone in x per channel, so each
// block's extreme maps to that block's max y -- exactly the max a pass over y finds
template <typename T, bool RELU>
__global__ __launch_bounds__(256) void bnq_absmax_mm_kernel(const float* __restrict__ xmm, int64_t nblk, int c,
                                                            int c_real, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, float* __restrict__ out) {
  // thread = one channel over a stride of the blocks (blockIdx.y): scale / shift read once
  float mx = 0.f;
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch < c_real) {
    const float sc = scale[ch], sh = shift[ch];
    for (int64_t b = blockIdx.y; b < nblk; b += gridDim.y) {
      // (y >= 0: its max sits at the block's extreme on scale's side, which xmm holds)
      const float v = fmaf(xmm[b * c + ch], sc, sh);
      mx = fmaxf(mx, to_f(from_f<T>(RELU ? fmaxf(v, 0.f) : v)));
    }
  }
  mx = wave_max(mx);
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}

// up to two activation quantizers of the same BatchNorm output (symbol/resnet_int8.py: a stage's first
// unit quantizes act1 once for conv1 and once for the shortcut conv, each with its own threshold state)
struct BnqTargets {
  void* out[2];
  int8_t* codes[2];
  float* unit[2];
  float qmax[2];
};
// NT: 1 = rn_set_tuning 18 bit 8's streaming hints, 4 = bit 64's write-through (sc1) stores
template <typename T, bool RELU, int NQ, int NT = 0>
__global__ __launch_bounds__(256) void bnq_codes_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, int64_t m, int c, int ct,
                                                        int64_t rows_per_block, BnqTargets tg,
                                                        const float* __restrict__ thr, int exact_div) {
  float t[NQ], unit[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    t[k] = thr[k];
    unit[k] = t[k] / tg.qmax[k];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *tg.unit[k] = unit[k];
  }
  const int tc = threadIdx.x % ct, tr = threadIdx.x / ct, rl = blockDim.x / ct;
  if (tr >= rl) return;
  const int cb = (blockIdx.x * ct + tc) * 16;
  const int64_t r0 = blockIdx.y * rows_per_block;
  const int64_t r1 = min(m, r0 + rows_per_block);
  constexpr int CE = 16 / sizeof(T);
  float sc[16], sh[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    sc[e] = scale[cb + e];
    sh[e] = shift[cb + e];
  }
  float inv[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) inv[k] = unit[k] > 0.f ? 1.f / unit[k] : 0.f;
  for (int64_t r = r0 + tr; r < r1; r += rl) {
    float f[16];
    bnq_load<T, RELU, (NT & 1) != 0>(x + r * c + cb, sc, sh, f);
    const int64_t off = r * c + cb;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      float g[16], tq[16], sm[16];
      uint32_t cw[4];
      // the quotient v / unit as v * (1 / unit): within 2^-22 |q| of the IEEE quotient, so the two
      // round alike unless the product lies that close to a half-integer -- then (rarely: checked per
      // wave) the exact division, so the codes stay those of round(v / unit) bit for bit (this kernel is
      // VALU-bound, and the division's ~11 instructions per element were a third of it).
      // Rounding: sm = tq + 1.5 * 2^23 rounds tq to the nearest integer (ties to even) in the low
      // mantissa bits -- the code's byte is sm's low byte, the integer sm - 1.5 * 2^23. That equals
      // roundf's (ties away) wherever tq is not within the near-half tolerance below, whose elements
      // take roundf of the exact quotient instead: |tq - rne(tq)| = 0.5 - |frac(tq) - 0.5|, so the test
      // is the same one, exactly
      constexpr float kMagic = 12582912.f;
      uint32_t nearm = exact_div ? 0xFFFFu : 0u;  // (rn_set_tuning 22 = 1: the division everywhere)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if constexpr (RELU) {  // (f >= 0, t >= 0: the clip is min(f, t), a select; tq >= 0)
          tq[e] = (f[e] < t[k] ? f[e] : t[k]) * inv[k];
          sm[e] = tq[e] + kMagic;
          // (the same test as below up to the rounding of its right-hand side, which the tolerance's 2x
          // margin over the reciprocal's error absorbs; a non-finite product fails the < and is exact)
          if (!(fabsf(tq[e] - (sm[e] - kMagic)) < fmaf(-4.8e-7f, tq[e], 0.5f))) nearm |= 1u << e;
        } else {
          tq[e] = fminf(fmaxf(f[e], -t[k]), t[k]) * inv[k];
          sm[e] = tq[e] + kMagic;
          const float d = fabsf(tq[e] - (sm[e] - kMagic));
          // (written as !(>) so that a non-finite product -- a unit so small its reciprocal overflows --
          // takes the exact path too)
          if (!(0.5f - d > fabsf(tq[e]) * 4.8e-7f)) nearm |= 1u << e;
        }
      }
      if (__any(nearm != 0u)) {
#pragma unroll
        for (int e = 0; e < 16; ++e)
          if ((nearm >> e) & 1u)
            sm[e] = (unit[k] > 0.f ? roundf(fminf(fmaxf(f[e], -t[k]), t[k]) / unit[k]) : 0.f) + kMagic;
      }
#pragma unroll
      for (int e = 0; e < 16; e += 4) {  // quant_codes_kernel's clip / round / dequantize
        const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(sm[e + 1]), __float_as_uint(sm[e]), 0x0c0c0400u);
        const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(sm[e + 3]), __float_as_uint(sm[e + 2]), 0x0c0c0400u);
        cw[e >> 2] = lo | (hi << 16);
#pragma unroll
        for (int u = 0; u < 4; ++u) g[e + u] = (sm[e + u] - kMagic) * unit[k];
      }
      if (tg.out[k])  // (null: codes only, the values expanded later by rn_quant_int8_expand)
#pragma unroll
        for (int h = 0; h < 16 / CE; ++h) {
          const uint4 o = f_to_chunk(g + h * CE, (const T*)nullptr);
          if constexpr ((NT & 4) != 0) {  // write-through: no dirty line left in the XCD L2 (as rn_bn.hip's st16)
            const bnq_u32x4 w = {o.x, o.y, o.z, o.w};
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(
                             reinterpret_cast<bnq_u32x4*>(reinterpret_cast<T*>(tg.out[k]) + off) + h),
                         "v"(w)
                         : "memory");
          } else if constexpr ((NT & 1) != 0) {  // the fake-quantized copy is read only by the weight gradients, later
            const bnq_u32x4 w = {o.x, o.y, o.z, o.w};
            __builtin_nontemporal_store(w, reinterpret_cast<bnq_u32x4*>(reinterpret_cast<T*>(tg.out[k]) + off) + h);
          } else {
            reinterpret_cast<uint4*>(reinterpret_cast<T*>(tg.out[k]) + off)[h] = o;
          }
        }
      if constexpr ((NT & 4) != 0) {
        const bnq_u32x4 w = {cw[0], cw[1], cw[2], cw[3]};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(tg.codes[k] + off), "v"(w) : "memory");
      } else {
        reinterpret_cast<uint4*>(tg.codes[k] + off)[0] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
      }
    }
  }
}
// ---- batched weight quantization (rn_weight_quant_pack): blockIdx.y = weight
__global__ __launch_bounds__(256) void wq_absmax_kernel(const rn_wquant_item* __restrict__ items,
                                                        float* __restrict__ curmax) {
  const rn_wquant_item it = items[blockIdx.y];
  const int64_t n = (int64_t)it.k * it.rs * it.c_real;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float m = 0.f;
  int64_t i0 = 0;
  if ((reinterpret_cast<uintptr_t>(it.master) & 15) == 0) {  // 16-byte chunks, then the tail
    const int64_t nc = n / 4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nc; i += stride) {
      const float4 v = reinterpret_cast<const float4*>(it.master)[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    i0 = nc * 4;
  }
  for (int64_t i = i0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    m = fmaxf(m, fabsf(it.master[i]));
  m = wave_max(m);
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned int*>(curmax + blockIdx.y),
              __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}
__global__ void wq_state_kernel(const rn_wquant_item* __restrict__ items, int count, float* __restrict__ ws) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  const rn_wquant_item it = items[j];
  const float t = quant_state_update(ws[j], it.minmax, 1, 1, 0.f, 0);
  ws[count + j] = t;
  ws[j] = 0.f;
  if (it.unit) it.unit[0] = t / (float)((1 << (it.nbits - 1)) - 1);
}
// One read of the master per weight: 64(k) x 64(c) tiles of one tap (as sgd_mom_pack_kernel), each
// element's q = round(w / unit) computed once; the fake-quantized copy and the int8 codes stored in
// master (KRSC) order, the data-gradient copy (CRSK) transposed through LDS so its rows are coalesced
// too. (The first form walked the CRSK copy in its own order, reading the master with a stride of
// RS*c_real floats per lane: 280 us per ResNet-50 step.) blockIdx.y = weight; blocks stride its tiles.
template <typename T>
__global__ __launch_bounds__(256) void wq_pack_kernel(const rn_wquant_item* __restrict__ items, int count,
                                                      const float* __restrict__ ws) {
  __shared__ float tile[64][65];
  const rn_wquant_item it = items[blockIdx.y];
  const float t = ws[count + blockIdx.y];
  const float qmax = (float)((1 << (it.nbits - 1)) - 1);
  const float unit = t / qmax;  // (quant_value's and the codes' unit)
  const int RS = it.rs, cr = it.c_real, K = it.k;
  const int kt = (K + 63) / 64, ct = (cr + 63) / 64;
  const int ntiles = kt * RS * ct;
  T* __restrict__ out = reinterpret_cast<T*>(it.w_crsk);
  const int cl = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  for (int tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
    const int c0 = (tl % ct) * 64, rest = tl / ct;
    const int tap = rest % RS, k0 = (rest / RS) * 64;
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {  // rows k0 + r, columns c0 + cl: coalesced over c
      const int r = r0 + 4 * j, k = k0 + r, ci = c0 + cl;
      if (k < K && ci < cr) {
        const int64_t kt_ = (int64_t)k * RS + tap;
        const float q = unit > 0.f ? roundf(it.master[kt_ * cr + ci] / unit) : 0.f;
        it.qw[kt_ * cr + ci] = q * unit;
        if (it.w_codes) it.w_codes[kt_ * it.c + ci] = (int8_t)(int)q;
        tile[r][cl] = q * unit;
      }
    }
    if (!out) continue;  // (uniform over the block)
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {  // rows c, columns k: coalesced over k
      const int r = r0 + 4 * j, ci = c0 + r, k = k0 + cl;
      if (k < K && ci < cr) out[((int64_t)ci * RS + tap) * it.k_pad + k] = from_f<T>(tile[cl][r]);
    }
    __syncthreads();
  }
}

// the threshold states of NQ quantizers of one tensor from its max (consumed and re-zeroed)
__global__ void quant_state_multi_kernel(float* __restrict__ curmax, float* minmax0, float* minmax1, int nq,
                                         int is_train, float decay0, float decay1, int first, float* __restrict__ thr) {
  thr[0] = quant_state_update(*curmax, minmax0, 0, is_train, decay0, first);
  if (nq > 1) thr[1] = quant_state_update(*curmax, minmax1, 0, is_train, decay1, first);
  *curmax = 0.f;
}

}  // namespace

int g_tune[RN_TUNE_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512, 0, 0, 0, 0, 0, 0, 0, 55, 0, 0, 50, 0, 0, 0, 0, 0, 0};

extern "C" {

const char* rn_last_error(void) { return g_last_error.c_str(); }

int rn_set_tuning(int32_t key, int32_t value) {
  RN_CHECK_ARG(key >= 0 && key < RN_TUNE_COUNT, "bad tuning key");
  RN_CHECK_ARG(kRnDiag || (key != RN_TUNE_DIAG_IGEMM_L1 && key != RN_TUNE_DIAG_WGRAD_NOEPI && key != RN_TUNE_IGEMM_SCHED) ||
                   value == 0,
               "diagnostic tuning key (3, 6, 7): only in the diagnostic build (RN_DIAG=1, librn_diag.so)");
  g_tune[key] = value;
  return 0;
}
int32_t rn_version(void) { return 100; }
#ifndef RN_BUILD_ID
#define RN_BUILD_ID "unknown"
#endif
// the marker prefix lets rn/build.py read the id from the file without loading it
static const char kBuildIdMarker[] = "RN_BUILD_ID=" RN_BUILD_ID;
const char* rn_build_id(void) { return kBuildIdMarker + 12; }
int32_t rn_device_cu_count(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
  return prop.multiProcessorCount;
}

int rn_pool_desc_init(rn_pool_desc* d) {
  RN_CHECK_ARG(d != nullptr, "null desc");
  RN_CHECK_ARG(d->dtype == RN_BF16 || d->dtype == RN_F32, "bad dtype");
  RN_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && d->c % 8 == 0, "bad shape");
  RN_CHECK_ARG(d->type == RN_POOL_MAX || d->type == RN_POOL_AVG, "bad pool type");
  if (d->global_pool) {
    d->r = d->h; d->s = d->w; d->stride_h = d->stride_w = 1; d->pad_h = d->pad_w = 0;
  }
  RN_CHECK_ARG(d->r > 0 && d->s > 0 && d->stride_h > 0 && d->stride_w > 0, "bad window");
  RN_CHECK_ARG(d->r * d->s <= 255, "window too large");
  d->p = (d->h + 2 * d->pad_h - d->r) / d->stride_h + 1;
  d->q = (d->w + 2 * d->pad_w - d->s) / d->stride_w + 1;
  RN_CHECK_ARG(d->p > 0 && d->q > 0, "empty output");
  return 0;
}

int rn_pool_fwd(const rn_pool_desc* d, const void* x, void* y, uint8_t* argmax, rn_stream_t stream) {
  return rn_pool_fwd_x(d, x, y, argmax, nullptr, nullptr, stream);
}

int rn_pool_fwd_x(const rn_pool_desc* d, const void* x, void* y, uint8_t* argmax, const float* in_scale,
                  const float* in_shift, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && y, "null argument");
  RN_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "in_scale / in_shift must both be set");
  PoolArgs a{d->n, d->h, d->w, d->c, d->r, d->s, d->stride_h, d->stride_w, d->pad_h, d->pad_w, d->p, d->q, d->type};
  a.fd_cpr = make_fastdiv(d->c / (d->dtype == RN_BF16 ? 8 : 4));
  a.fd_a = make_fastdiv(d->q);
  a.fd_b = make_fastdiv(d->p);
  RN_CHECK_ARG((int64_t)d->n * d->h * d->w * d->c < INT32_MAX, "pooling tensor exceeds 2^31 elements");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)d->n * d->p * d->q * d->c / 8;
  if (d->dtype == RN_BF16) {
    if (in_scale)
      hipLaunchKernelGGL((pool_fwd_kernel<bf16_t, true>), dim3(grid1d(total)), dim3(256), 0, st, a, (const bf16_t*)x,
                         (bf16_t*)y, argmax, in_scale, in_shift);
    else
      hipLaunchKernelGGL(pool_fwd_kernel<bf16_t>, dim3(grid1d(total)), dim3(256), 0, st, a, (const bf16_t*)x,
                         (bf16_t*)y, argmax, nullptr, nullptr);
  } else if (in_scale) {
    hipLaunchKernelGGL((pool_fwd_kernel<float, true>), dim3(grid1d(total * 2)), dim3(256), 0, st, a, (const float*)x,
                       (float*)y, argmax, in_scale, in_shift);
  } else {
    hipLaunchKernelGGL(pool_fwd_kernel<float>, dim3(grid1d(total * 2)), dim3(256), 0, st, a, (const float*)x,
                       (float*)y, argmax, nullptr, nullptr);
  }
  return rn_check_launch("pool_fwd");
}

}  // extern "C" (reopened below, after the 2x2-block max-pool backward)

namespace {
// Max pool 3x3 / stride 2 / pad 1 with H = 2P, W = 2Q (the ResNet stem pool, symbol/resnet.py:97),
// backward: thread per (image, 2x2 input block (2i.., 2j..), channel chunk). The block's pixels take
// gradient only from the outputs (i | i+1) x (j | j+1) -- input row 2i from output row i, row 2i+1
// from rows i and i+1 -- so each dy / tap-index chunk is read once per block instead of once per
// covered input pixel (up to 4x). Sums in the generic kernel's order (outputs row-major): bit-identical.
// RED (bf16, the stem's bn0 -> relu0 -> pool, symbol/resnet.py:94-97): the pool backward completes the
// BatchNorm+ReLU output gradient, so it also reduces that BN's backward as the conv epilogues do
// (igemm_big_kernel EPI 2): sum dz, sum dz*(x - mean), dz = dx * relu'(x sc + sh) on the stored dx ->
// part[block][C][2]. A thread keeps one channel chunk (C / 8 divides the 256-thread block), the lanes
// of a chunk then the block's waves are summed in a fixed order.
struct PoolRed {
  const bf16_t* bn_x;
  const float *mean, *sc, *sh;
  float* part;
  int relu;
};
constexpr int kPoolRedMaxC = 256;
template <typename T, bool RED = false>
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(PoolArgs a, const T* __restrict__ dy,
                                                             const uint8_t* __restrict__ argmax, T* __restrict__ dx,
                                                             const T* __restrict__ add, PoolRed rd) {
  constexpr int CE = 16 / sizeof(T);
  const int cpr = a.c / CE;
  const uint32_t total = (uint32_t)a.n * a.p * a.q * cpr;  // blocks x chunks (P = H/2, Q = W/2)
  float s1[RED ? 8 : 1], s2[RED ? 8 : 1], r_mu[RED ? 8 : 1], r_sc[RED ? 8 : 1], r_sh[RED ? 8 : 1];
  if constexpr (RED) {
    const int c0 = (int)(threadIdx.x % cpr) * 8;  // (the chunk of every i this thread visits)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = s2[e] = 0.f;
      r_mu[e] = rd.mean[c0 + e];
      r_sc[e] = rd.sc[c0 + e];
      r_sh[e] = rd.sh[c0 + e];
    }
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t blk = fdiv(i, a.fd_cpr);
    const int cc = (int)(i - blk * cpr);
    const uint32_t t = fdiv(blk, a.fd_a);  // fd_a: q
    const int bj = (int)(blk - t * a.q);
    const uint32_t n = fdiv(t, a.fd_b);    // fd_b: p
    const int bi = (int)(t - n * a.p);
    uint4 g4[4];
    uint64_t am4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // outputs (bi + u/2, bj + u%2)
      const int pp = bi + (u >> 1), qq = bj + (u & 1);
      const bool ok = pp < a.p && qq < a.q;
      const int64_t ob = (((int64_t)n * a.p + (ok ? pp : bi)) * a.q + (ok ? qq : bj)) * a.c + cc * CE;
      g4[u] = ok ? *reinterpret_cast<const uint4*>(dy + ob) : make_uint4(0, 0, 0, 0);
      am4[u] = !ok ? ~0ull : CE == 8 ? *reinterpret_cast<const uint64_t*>(argmax + ob)
                                     : (uint64_t)*reinterpret_cast<const uint32_t*>(argmax + ob);
    }
    float g[4][CE];
#pragma unroll
    for (int u = 0; u < 4; ++u) chunk_to_f(g4[u], g[u], (const T*)nullptr);
#pragma unroll
    for (int v = 0; v < 4; ++v) {  // input pixel (2 bi + dh, 2 bj + dw)
      const int dh = v >> 1, dw = v & 1;
      const int64_t xi = (((int64_t)n * a.h + 2 * bi + dh) * a.w + 2 * bj + dw) * cpr + cc;
      float acc[CE];
      if (add) chunk_to_f(reinterpret_cast<const uint4*>(add)[xi], acc, (const T*)nullptr);
      else
#pragma unroll
        for (int e = 0; e < CE; ++e) acc[e] = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int du = u >> 1, dv = u & 1;  // output (bi + du, bj + dv)
        if ((du && !dh) || (dv && !dw)) continue;  // row 2 bi is only in output row bi (same for columns)
        const int tap = (dh + 1 - 2 * du) * 3 + (dw + 1 - 2 * dv);
#pragma unroll
        for (int e = 0; e < CE; ++e)
          if ((int)((am4[u] >> (8 * e)) & 0xFF) == tap) acc[e] += g[u][e];
      }
      const uint4 o = f_to_chunk(acc, (const T*)nullptr);
      reinterpret_cast<uint4*>(dx)[xi] = o;
      if constexpr (RED) {  // on the stored (rounded) values, as a separate pass would read them
        float g[8], xv[8];
        chunk_to_f(o, g, (const bf16_t*)nullptr);
        chunk_to_f(reinterpret_cast<const uint4*>(rd.bn_x)[xi], xv, (const bf16_t*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = (!rd.relu || fmaf(xv[e], r_sc[e], r_sh[e]) > 0.f) ? g[e] : 0.f;
          s1[e] += dz;
          s2[e] = fmaf(dz, xv[e] - r_mu[e], s2[e]);
        }
      }
    }
  }
  if constexpr (RED) {
    __shared__ float red[4][2][kPoolRedMaxC];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int o = cpr; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (lane < cpr)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wid][0][lane * 8 + e] = s1[e];
        red[wid][1][lane * 8 + e] = s2[e];
      }
    __syncthreads();
    for (int c = threadIdx.x; c < a.c; c += blockDim.x) {
      float* dst = rd.part + ((int64_t)blockIdx.x * a.c + c) * 2;
      dst[0] = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
      dst[1] = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    }
  }
}
// the 2x2-block form applies (and, bf16 with C / 8 dividing 256 and C <= kPoolRedMaxC, its BN reduction)
bool maxpool3s2_ok(const rn_pool_desc* d) {
  return d->type == RN_POOL_MAX && d->r == 3 && d->s == 3 && d->stride_h == 2 && d->stride_w == 2 && d->pad_h == 1 &&
         d->pad_w == 1 && d->h == 2 * d->p && d->w == 2 * d->q && g_tune[RN_TUNE_POOL_BLOCK_BWD] != 1;
}
bool pool_red_ok(const rn_pool_desc* d) {
  return d && maxpool3s2_ok(d) && d->dtype == RN_BF16 && d->c <= kPoolRedMaxC && 256 % (d->c / 8) == 0;
}
int pool_red_blocks(const rn_pool_desc* d) {  // (grid-stride: at most 1024 workgroups, one partial each)
  return grid1d((int64_t)d->n * d->p * d->q * d->c / 8, 256, 1024);
}
}  // namespace

extern "C" {
namespace {
int pool_bwd(const rn_pool_desc* d, const void* dy, const uint8_t* argmax, void* dx, const void* add_src,
             const PoolRed* red, rn_stream_t stream) {
  RN_CHECK_ARG(d && dy && dx, "null argument");
  RN_CHECK_ARG(d->type != RN_POOL_MAX || argmax, "max pool backward needs argmax");
  PoolArgs a{d->n, d->h, d->w, d->c, d->r, d->s, d->stride_h, d->stride_w, d->pad_h, d->pad_w, d->p, d->q, d->type};
  a.fd_cpr = make_fastdiv(d->c / (d->dtype == RN_BF16 ? 8 : 4));
  a.fd_a = make_fastdiv(d->w);
  a.fd_b = make_fastdiv(d->h);
  RN_CHECK_ARG((int64_t)d->n * d->h * d->w * d->c < INT32_MAX, "pooling tensor exceeds 2^31 elements");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)d->n * d->h * d->w * d->c / 8;
  if (maxpool3s2_ok(d)) {
    PoolArgs b = a;
    b.fd_a = make_fastdiv(d->q);
    b.fd_b = make_fastdiv(d->p);
    const int64_t nb = (int64_t)d->n * d->p * d->q * d->c / (d->dtype == RN_BF16 ? 8 : 4);
    if (red && red->part)
      hipLaunchKernelGGL((maxpool3s2_bwd_kernel<bf16_t, true>), dim3(pool_red_blocks(d)), dim3(256), 0, st, b,
                         (const bf16_t*)dy, argmax, (bf16_t*)dx, (const bf16_t*)add_src, *red);
    else if (d->dtype == RN_BF16)
      hipLaunchKernelGGL(maxpool3s2_bwd_kernel<bf16_t>, dim3(grid1d(nb)), dim3(256), 0, st, b, (const bf16_t*)dy,
                         argmax, (bf16_t*)dx, (const bf16_t*)add_src, PoolRed{});
    else
      hipLaunchKernelGGL(maxpool3s2_bwd_kernel<float>, dim3(grid1d(nb)), dim3(256), 0, st, b, (const float*)dy,
                         argmax, (float*)dx, (const float*)add_src, PoolRed{});
    return rn_check_launch("maxpool3s2_bwd");
  }
  RN_CHECK_ARG(!(red && red->part), "pool BN reduction: the 3x3 / stride-2 max pool with H = 2P, W = 2Q only");
  if (d->dtype == RN_BF16)
    hipLaunchKernelGGL(pool_bwd_kernel<bf16_t>, dim3(grid1d(total)), dim3(256), 0, st, a, (const bf16_t*)dy,
                       argmax, (bf16_t*)dx, (const bf16_t*)add_src);
  else
    hipLaunchKernelGGL(pool_bwd_kernel<float>, dim3(grid1d(total * 2)), dim3(256), 0, st, a, (const float*)dy,
                       argmax, (float*)dx, (const float*)add_src);
  return rn_check_launch("pool_bwd");
}
}  // namespace

int rn_pool_bwd(const rn_pool_desc* d, const void* dy, const uint8_t* argmax, void* dx, const void* add_src,
                rn_stream_t stream) {
  return pool_bwd(d, dy, argmax, dx, add_src, nullptr, stream);
}

int64_t rn_pool_bwd_bnred_blocks(const rn_pool_desc* d) { return pool_red_ok(d) ? pool_red_blocks(d) : 0; }

int rn_pool_bwd_bnred(const rn_pool_desc* d, const void* dy, const uint8_t* argmax, void* dx, const void* add_src,
                      const void* bn_x, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                      int32_t relu, float* part, rn_stream_t stream) {
  RN_CHECK_ARG(d && bn_x && bn_mean && bn_scale && bn_shift && part, "null argument");
  RN_CHECK_ARG(pool_red_ok(d), "pool BN reduction: bf16 3x3 / stride-2 max pool, H = 2P, W = 2Q, C / 8 dividing 256");
  const PoolRed r{(const bf16_t*)bn_x, bn_mean, bn_scale, bn_shift, part, relu};
  return pool_bwd(d, dy, argmax, dx, add_src, &r, stream);
}

int rn_softmax_output(int32_t grad_dtype, int32_t batch, int32_t ncls, int32_t ld, const float* logits,
                      const float* label, float* prob, void* dlogits, float grad_scale, float* stats,
                      rn_stream_t stream) {
  RN_CHECK_ARG(logits && label && batch > 0 && ncls > 0 && ld >= ncls, "bad arguments");
  hipStream_t st = as_stream(stream);
  const int rows_per_block = 4;
  dim3 grid((batch + rows_per_block - 1) / rows_per_block);
  if (grad_dtype == RN_BF16)
    hipLaunchKernelGGL(softmax_output_kernel<bf16_t>, grid, dim3(256), 0, st, batch, ncls, ld, logits, label, prob,
                       (bf16_t*)dlogits, grad_scale, stats);
  else
    hipLaunchKernelGGL(softmax_output_kernel<float>, grid, dim3(256), 0, st, batch, ncls, ld, logits, label, prob,
                       (float*)dlogits, grad_scale, stats);
  return rn_check_launch("softmax_output");
}

int rn_col_sum(int32_t dtype, int64_t m, int32_t c, int32_t ld, const void* x, float* out, int32_t accumulate,
               rn_stream_t stream) {
  RN_CHECK_ARG(x && out && m > 0 && c > 0 && ld >= c, "bad arguments");
  hipStream_t st = as_stream(stream);
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(col_sum_kernel<bf16_t>, dim3(c), dim3(256), 0, st, m, c, ld, (const bf16_t*)x, out, accumulate);
  else
    hipLaunchKernelGGL(col_sum_kernel<float>, dim3(c), dim3(256), 0, st, m, c, ld, (const float*)x, out, accumulate);
  return rn_check_launch("col_sum");
}

int rn_sgd_mom_update(int32_t ntensors, const int64_t* offsets, const int64_t* numels, const float* wds, float* w,
                      const float* g, float* mom, void* w_lowp, int32_t lowp_dtype, float lr, const float* lr_dev,
                      float momentum, float rescale_grad, float clip, rn_stream_t stream) {
  RN_CHECK_ARG(ntensors > 0 && offsets && numels && wds && w && g && mom, "bad arguments");
  RN_CHECK_ARG(ntensors <= 65535, "too many tensors");
  hipStream_t st = as_stream(stream);
  dim3 grid(64, ntensors);
  if (w_lowp && lowp_dtype == RN_BF16)
    hipLaunchKernelGGL(sgd_mom_kernel<bf16_t>, grid, dim3(256), 0, st, offsets, numels, wds, w, g, mom,
                       (bf16_t*)w_lowp, lr, lr_dev, momentum, rescale_grad, clip);
  else
    hipLaunchKernelGGL(sgd_mom_kernel<float>, grid, dim3(256), 0, st, offsets, numels, wds, w, g, mom,
                       (float*)w_lowp, lr, lr_dev, momentum, rescale_grad, clip);
  return rn_check_launch("sgd_mom_update");
}

int rn_sgd_mom_update_pack(int32_t ntensors, const int64_t* offsets, const int64_t* numels, const float* wds,
                           float* w, const float* g, float* mom, const rn_wpack* packs, const int32_t* work,
                           int32_t nwork, int32_t lowp_dtype, float lr, const float* lr_dev, float momentum,
                           float rescale_grad, float clip, rn_stream_t stream) {
  RN_CHECK_ARG(ntensors > 0 && offsets && numels && wds && w && g && mom && packs && work && nwork > 0,
               "bad arguments");
  hipStream_t st = as_stream(stream);
  const int4* wk = reinterpret_cast<const int4*>(work);
  if (lowp_dtype == RN_BF16)
    hipLaunchKernelGGL(sgd_mom_pack_kernel<bf16_t>, dim3(nwork), dim3(256), 0, st, offsets, wds, w, g, mom, packs, wk,
                       numels, lr, lr_dev, momentum, rescale_grad, clip);
  else
    hipLaunchKernelGGL(sgd_mom_pack_kernel<float>, dim3(nwork), dim3(256), 0, st, offsets, wds, w, g, mom, packs, wk,
                       numels, lr, lr_dev, momentum, rescale_grad, clip);
  return rn_check_launch("sgd_mom_update_pack");
}

#if RN_DIAG
// Diagnostic: the same kernel with every global index checked against lim = {nparam, then per
// tensor KRSC and CRSK copy sizes}; out-of-range accesses are skipped and flagged in *flag.
int rn_sgd_mom_update_pack_checked(int32_t ntensors, const int64_t* offsets, const int64_t* numels, const float* wds,
                                   float* w, const float* g, float* mom, const rn_wpack* packs, const int32_t* work,
                                   int32_t nwork, int32_t lowp_dtype, float lr, float momentum, float rescale_grad,
                                   const int64_t* lim, int32_t* flag, rn_stream_t stream) {
  RN_CHECK_ARG(ntensors > 0 && nwork > 0 && lim && flag, "bad arguments");
  hipStream_t st = as_stream(stream);
  const int4* wk = reinterpret_cast<const int4*>(work);
  if (lowp_dtype == RN_BF16)
    hipLaunchKernelGGL((sgd_mom_pack_kernel<bf16_t, true>), dim3(nwork), dim3(256), 0, st, offsets, wds, w, g, mom,
                       packs, wk, numels, lr, nullptr, momentum, rescale_grad, -1.f, lim, flag);
  else
    hipLaunchKernelGGL((sgd_mom_pack_kernel<float, true>), dim3(nwork), dim3(256), 0, st, offsets, wds, w, g, mom,
                       packs, wk, numels, lr, nullptr, momentum, rescale_grad, -1.f, lim, flag);
  return rn_check_launch("sgd_mom_update_pack_checked");
}
#endif  // RN_DIAG

int32_t rn_sgd_pack_work(int32_t ntensors, const int64_t* numels, const rn_wpack* packs, int32_t* work,
                         int32_t max_items) {
  RN_CHECK_ARG(ntensors > 0 && numels && packs && work, "bad arguments");
  int32_t n = 0;
  auto put = [&](int a, int b, int c, int d) {
    if (n < max_items) {
      work[4 * n] = a;
      work[4 * n + 1] = b;
      work[4 * n + 2] = c;
      work[4 * n + 3] = d;
    }
    ++n;
  };
  for (int t = 0; t < ntensors; ++t) {
    const rn_wpack& p = packs[t];
    if (p.crsk) {
      RN_CHECK_ARG((int64_t)p.k * p.rs * p.creal == numels[t], "pack table does not match the tensor size");
      for (int k0 = 0; k0 < p.k; k0 += 64)
        for (int tap = 0; tap < p.rs; ++tap)
          for (int c0 = 0; c0 < p.creal; c0 += 64) put(t, k0, tap, c0);
    } else {
      RN_CHECK_ARG(numels[t] < (int64_t)1 << 31, "tensor too large");
      for (int64_t s = 0; s < numels[t]; s += kSgdChunk) put(t, (int)s, 0, 0);
    }
  }
  RN_CHECK_ARG(n <= max_items, "work table too small");
  return n;
}

int rn_nchw_to_nhwc(int32_t n, int32_t c, int32_t h, int32_t w, int32_t c_pad, const float* src, void* dst,
                    int32_t dst_dtype, rn_stream_t stream) {
  RN_CHECK_ARG(src && dst && c_pad >= c, "bad arguments");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)n * h * w * c_pad;
  if (dst_dtype == RN_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, dim3(grid1d(total)), dim3(256), 0, st, n, c, h, w, c_pad, src,
                       (bf16_t*)dst);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid1d(total)), dim3(256), 0, st, n, c, h, w, c_pad, src,
                       (float*)dst);
  return rn_check_launch("nchw_to_nhwc");
}

int rn_cast(int64_t n, const void* src, int32_t sd, void* dst, int32_t dd, rn_stream_t stream) {
  RN_CHECK_ARG(src && dst && n >= 0, "bad arguments");
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  dim3 g(grid1d(n)), b(256);
  if (sd == RN_F32 && dd == RN_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), g, b, 0, st, n, (const float*)src, (bf16_t*)dst);
  else if (sd == RN_BF16 && dd == RN_F32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), g, b, 0, st, n, (const bf16_t*)src, (float*)dst);
  else if (sd == RN_F32 && dd == RN_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, b, 0, st, n, (const float*)src, (float*)dst);
  else
    hipLaunchKernelGGL((cast_kernel<bf16_t, bf16_t>), g, b, 0, st, n, (const bf16_t*)src, (bf16_t*)dst);
  return rn_check_launch("cast");
}

int rn_eltwise_add(int64_t n, int32_t dtype, const void* a, const void* b, void* dst, int32_t relu,
                   rn_stream_t stream) {
  RN_CHECK_ARG(a && dst && n >= 0, "bad arguments");
  const int CE = dtype == RN_BF16 ? 8 : 4;
  RN_CHECK_ARG(n % CE == 0, "n must be a multiple of the 16-byte chunk");
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int64_t nc = n / CE;
  dim3 g(grid1d(nc)), bl(256);
  if (dtype == RN_BF16) {
    if (relu) hipLaunchKernelGGL((add_kernel<bf16_t, true>), g, bl, 0, st, nc, (const bf16_t*)a, (const bf16_t*)b, (bf16_t*)dst);
    else hipLaunchKernelGGL((add_kernel<bf16_t, false>), g, bl, 0, st, nc, (const bf16_t*)a, (const bf16_t*)b, (bf16_t*)dst);
  } else {
    if (relu) hipLaunchKernelGGL((add_kernel<float, true>), g, bl, 0, st, nc, (const float*)a, (const float*)b, (float*)dst);
    else hipLaunchKernelGGL((add_kernel<float, false>), g, bl, 0, st, nc, (const float*)a, (const float*)b, (float*)dst);
  }
  return rn_check_launch("eltwise_add");
}

int rn_relu_bwd(int64_t n, int32_t dtype, const void* y, const void* dy, void* dx, const void* add_src,
                rn_stream_t stream) {
  RN_CHECK_ARG(y && dy && dx && n >= 0, "bad arguments");
  const int CE = dtype == RN_BF16 ? 8 : 4;
  RN_CHECK_ARG(n % CE == 0, "n must be a multiple of the 16-byte chunk");
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int64_t nc = n / CE;
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(relu_bwd_kernel<bf16_t>, dim3(grid1d(nc)), dim3(256), 0, st, nc, (const bf16_t*)y,
                       (const bf16_t*)dy, (bf16_t*)dx, (const bf16_t*)add_src);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(grid1d(nc)), dim3(256), 0, st, nc, (const float*)y,
                       (const float*)dy, (float*)dx, (const float*)add_src);
  return rn_check_launch("relu_bwd");
}

}  // extern "C"

// rn_quant_int8_fwd; unit (nullable) also receives t / qmax
static int quant_fwd_values(int32_t dtype, int64_t n, const void* x, void* out, float* minmax, int32_t is_weight,
                            int32_t is_train, float ema_decay, int32_t first_batch, int32_t nbits, float* ws,
                            float* unit, rn_stream_t stream) {
  RN_CHECK_ARG(x && out && ws && n > 0, "bad arguments");
  RN_CHECK_ARG(is_weight || minmax, "activation quantization needs the minmax state");
  RN_CHECK_ARG(nbits >= 2 && nbits <= 16, "bad nbits");
  hipStream_t st = as_stream(stream);
  const float qmax = (float)((1 << (nbits - 1)) - 1);
  float* curmax = ws;  // zero on entry (left zero by the state kernel)
  float* thr = ws + 1;
  const bool need_max = is_weight || is_train;
  if (need_max) {
    if (dtype == RN_BF16)
      hipLaunchKernelGGL(absmax_kernel<bf16_t>, dim3(grid1d(n / 8, 256, 1024)), dim3(256), 0, st, n, (const bf16_t*)x,
                         curmax);
    else
      hipLaunchKernelGGL(absmax_kernel<float>, dim3(grid1d(n / 4, 256, 1024)), dim3(256), 0, st, n, (const float*)x,
                         curmax);
  }
  hipLaunchKernelGGL(quant_state_kernel, dim3(1), dim3(1), 0, st, curmax, minmax, is_weight, is_train, ema_decay,
                     first_batch, thr, qmax, unit);
  const int clip = is_weight ? 0 : 1;
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(quant_apply_kernel<bf16_t>, dim3(grid1d(n)), dim3(256), 0, st, n, (const bf16_t*)x,
                       (bf16_t*)out, thr, qmax, clip);
  else
    hipLaunchKernelGGL(quant_apply_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st, n, (const float*)x,
                       (float*)out, thr, qmax, clip);
  return rn_check_launch("quant_int8_fwd");
}

extern "C" {

int rn_quant_int8_fwd(int32_t dtype, int64_t n, const void* x, void* out, float* minmax, int32_t is_weight,
                      int32_t is_train, float ema_decay, int32_t first_batch, int32_t nbits, float* ws,
                      rn_stream_t stream) {
  return quant_fwd_values(dtype, n, x, out, minmax, is_weight, is_train, ema_decay, first_batch, nbits, ws, nullptr,
                          stream);
}

int rn_quant_int8_fwd_codes(int32_t dtype, int64_t n, const void* x, void* out, void* codes, float* unit,
                            float* minmax, int32_t is_weight, int32_t is_train, float ema_decay, int32_t first_batch,
                            int32_t nbits, float* ws, rn_stream_t stream) {
  RN_CHECK_ARG(x && ws && unit && n > 0 && (out || codes), "bad arguments");
  RN_CHECK_ARG(nbits >= 2 && nbits <= 8, "int8 codes need nbits <= 8");
  RN_CHECK_ARG(!codes || n % 16 == 0, "int8 codes: n must be a multiple of 16");
  if (!codes) {  // the fake-quantized values (and the unit) only
    return quant_fwd_values(dtype, n, x, out, minmax, is_weight, is_train, ema_decay, first_batch, nbits, ws, unit,
                            stream);
  }
  RN_CHECK_ARG(is_weight || minmax, "activation quantization needs the minmax state");
  hipStream_t st = as_stream(stream);
  const float qmax = (float)((1 << (nbits - 1)) - 1);
  float* curmax = ws;  // zero on entry (left zero by the state kernel)
  float* thr = ws + 1;
  if (is_weight || is_train) {
    if (dtype == RN_BF16)
      hipLaunchKernelGGL(absmax_kernel<bf16_t>, dim3(grid1d(n / 8, 256, 1024)), dim3(256), 0, st, n, (const bf16_t*)x,
                         curmax);
    else
      hipLaunchKernelGGL(absmax_kernel<float>, dim3(grid1d(n / 4, 256, 1024)), dim3(256), 0, st, n, (const float*)x,
                         curmax);
  }
  hipLaunchKernelGGL(quant_state_kernel, dim3(1), dim3(1), 0, st, curmax, minmax, is_weight, is_train, ema_decay,
                     first_batch, thr, qmax, nullptr);
  const int clip = is_weight ? 0 : 1;
  const int64_t nc = n / 16;
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(quant_codes_kernel<bf16_t>, dim3(grid1d(nc)), dim3(256), 0, st, nc, (const bf16_t*)x,
                       (bf16_t*)out, (int8_t*)codes, thr, qmax, clip, unit);
  else
    hipLaunchKernelGGL(quant_codes_kernel<float>, dim3(grid1d(nc)), dim3(256), 0, st, nc, (const float*)x,
                       (float*)out, (int8_t*)codes, thr, qmax, clip, unit);
  return rn_check_launch("quant_int8_fwd_codes");
}

extern "C++" {
template <typename T, bool RELU, int NQ>
static void launch_quant_codes_bn(const rn_bn_desc* d, const void* x, const float* scale, const float* shift,
                                  const BnqTargets& tg, float* const* minmax, const float* decay, float* ws,
                                  int32_t is_train, int32_t first_batch, hipStream_t st) {
  float* curmax = ws;  // zero on entry (left zero by the state kernel)
  float* thr = ws + 1;
  const int cpr = d->c / 16;  // 16-channel groups per row
  int ct = std::min(cpr, 64);
  while (cpr % ct) --ct;
  const int rl = 256 / ct, gx = cpr / ct;
  auto geo = [&](int rows_each) {
    const int64_t want = std::max<int64_t>(1, 4096 / gx);
    const int64_t maxrb = std::max<int64_t>(1, d->m / ((int64_t)rl * rows_each));
    const int nrb = (int)std::min(want, maxrb);
    return std::make_pair(nrb, (d->m + nrb - 1) / nrb);
  };
  if (is_train && d->xmm && RELU) {  // one max for all the quantizers of the tensor: the producer's block extremes
    const int gx = (d->c_real + 255) / 256;
    const int gy = (int)std::max<int64_t>(1, std::min<int64_t>(d->xmm_blocks, std::max(1, 512 / gx)));
    hipLaunchKernelGGL((bnq_absmax_mm_kernel<T, RELU>), dim3(gx, gy), dim3(256), 0, st, d->xmm, d->xmm_blocks, d->c,
                       d->c_real, scale, shift, curmax);
  } else if (is_train) {  // ... or from a pass over x
    const auto g = geo(16);
    hipLaunchKernelGGL((bnq_absmax_kernel<T, RELU>), dim3(gx, g.first), dim3(256), 0, st, (const T*)x, scale, shift,
                       d->m, d->c, ct, g.second, curmax);
  }
  hipLaunchKernelGGL(quant_state_multi_kernel, dim3(1), dim3(1), 0, st, curmax, minmax[0], minmax[NQ - 1], NQ,
                     is_train, decay[0], decay[NQ - 1], first_batch, thr);
  const auto g = geo(8);
  if (g_tune[RN_TUNE_BN_NT] & 64)
    hipLaunchKernelGGL((bnq_codes_kernel<T, RELU, NQ, 4>), dim3(gx, g.first), dim3(256), 0, st, (const T*)x, scale,
                       shift, d->m, d->c, ct, g.second, tg, thr, g_tune[RN_TUNE_QUANT_DIV] == 1 ? 1 : 0);
  else if (g_tune[RN_TUNE_BN_NT] & 8)
    hipLaunchKernelGGL((bnq_codes_kernel<T, RELU, NQ, 1>), dim3(gx, g.first), dim3(256), 0, st, (const T*)x, scale,
                       shift, d->m, d->c, ct, g.second, tg, thr, g_tune[RN_TUNE_QUANT_DIV] == 1 ? 1 : 0);
  else
    hipLaunchKernelGGL((bnq_codes_kernel<T, RELU, NQ>), dim3(gx, g.first), dim3(256), 0, st, (const T*)x, scale,
                       shift, d->m, d->c, ct, g.second, tg, thr, g_tune[RN_TUNE_QUANT_DIV] == 1 ? 1 : 0);
}
template <int NQ>
static int quant_codes_bn(const rn_bn_desc* d, const void* x, const float* scale, const float* shift,
                          const BnqTargets& tg, float* const* minmax, const float* decay, float* ws, int32_t is_train,
                          int32_t first_batch, hipStream_t st) {
  RN_CHECK_ARG(d && x && scale && shift && ws, "null argument");
  RN_CHECK_ARG(d->dtype == RN_BF16 || d->dtype == RN_F32, "bad dtype");
  RN_CHECK_ARG(d->m > 0 && d->c > 0 && d->c % 16 == 0, "bad shape (c must be a multiple of 16)");
  for (int k = 0; k < NQ; ++k) RN_CHECK_ARG(tg.codes[k] && tg.unit[k] && minmax[k], "null argument");
  const bool bf = d->dtype == RN_BF16;
  if (d->relu) {
    if (bf) launch_quant_codes_bn<bf16_t, true, NQ>(d, x, scale, shift, tg, minmax, decay, ws, is_train, first_batch, st);
    else launch_quant_codes_bn<float, true, NQ>(d, x, scale, shift, tg, minmax, decay, ws, is_train, first_batch, st);
  } else {
    if (bf) launch_quant_codes_bn<bf16_t, false, NQ>(d, x, scale, shift, tg, minmax, decay, ws, is_train, first_batch, st);
    else launch_quant_codes_bn<float, false, NQ>(d, x, scale, shift, tg, minmax, decay, ws, is_train, first_batch, st);
  }
  return rn_check_launch("quant_int8_fwd_codes_bn");
}
}  // extern "C++"

int rn_quant_int8_fwd_codes_bn(const rn_bn_desc* d, const void* x, const float* scale, const float* shift, void* out,
                               void* codes, float* unit, float* minmax, int32_t is_train, float ema_decay,
                               int32_t first_batch, int32_t nbits, float* ws, rn_stream_t stream) {
  RN_CHECK_ARG(nbits >= 2 && nbits <= 8, "int8 codes need nbits <= 8");
  BnqTargets tg{{out, nullptr}, {(int8_t*)codes, nullptr}, {unit, nullptr}, {(float)((1 << (nbits - 1)) - 1), 1.f}};
  float* mm[2] = {minmax, nullptr};
  const float decay[2] = {ema_decay, 0.f};
  return quant_codes_bn<1>(d, x, scale, shift, tg, mm, decay, ws, is_train, first_batch, as_stream(stream));
}

int rn_quant_int8_fwd_codes_bn2(const rn_bn_desc* d, const void* x, const float* scale, const float* shift,
                                void* out, void* codes, float* unit, float* minmax, float ema_decay, int32_t nbits,
                                void* out2, void* codes2, float* unit2, float* minmax2, float ema_decay2,
                                int32_t nbits2, int32_t is_train, int32_t first_batch, float* ws, rn_stream_t stream) {
  RN_CHECK_ARG(nbits >= 2 && nbits <= 8 && nbits2 >= 2 && nbits2 <= 8, "int8 codes need nbits <= 8");
  BnqTargets tg{{out, out2}, {(int8_t*)codes, (int8_t*)codes2}, {unit, unit2},
                {(float)((1 << (nbits - 1)) - 1), (float)((1 << (nbits2 - 1)) - 1)}};
  float* mm[2] = {minmax, minmax2};
  const float decay[2] = {ema_decay, ema_decay2};
  return quant_codes_bn<2>(d, x, scale, shift, tg, mm, decay, ws, is_train, first_batch, as_stream(stream));
}

int rn_quant_int8_expand(int32_t dtype, int64_t n, const void* codes, const float* unit, void* out,
                         rn_stream_t stream) {
  RN_CHECK_ARG(codes && unit && out && n > 0 && n % 16 == 0, "bad arguments (n a multiple of 16)");
  RN_CHECK_ARG(((uintptr_t)codes & 15) == 0 && ((uintptr_t)out & 15) == 0, "16-byte aligned codes / out");
  const int64_t nc = n / 16;
  hipStream_t st = as_stream(stream);
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(quant_expand_kernel<bf16_t>, dim3(grid1d(nc)), dim3(256), 0, st, nc, (const int8_t*)codes, unit,
                       (bf16_t*)out);
  else if (dtype == RN_F32)
    hipLaunchKernelGGL(quant_expand_kernel<float>, dim3(grid1d(nc)), dim3(256), 0, st, nc, (const int8_t*)codes, unit,
                       (float*)out);
  else
    RN_CHECK_ARG(false, "bad dtype");
  return rn_check_launch("quant_int8_expand");
}

int rn_weight_quant_pack(const rn_wquant_item* items, int32_t count, int32_t dtype, float* ws,
                         rn_stream_t stream) {
  RN_CHECK_ARG(items && ws && count > 0 && count <= 65535, "bad arguments");
  RN_CHECK_ARG(dtype == RN_BF16 || dtype == RN_F32, "bad dtype");
  hipStream_t st = as_stream(stream);
  // ws is the quantizers' shared workspace: the activation quantizers leave their thresholds in
  // ws[1..2], so the per-weight max accumulators are cleared here, not assumed zero
  if (hipMemsetAsync(ws, 0, sizeof(float) * (size_t)count, st) != hipSuccess) return rn_check_launch("weight_quant_pack");
  hipLaunchKernelGGL(wq_absmax_kernel, dim3(64, count), dim3(256), 0, st, items, ws);
  hipLaunchKernelGGL(wq_state_kernel, dim3((count + 63) / 64), dim3(64), 0, st, items, count, ws);
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(wq_pack_kernel<bf16_t>, dim3(256, count), dim3(256), 0, st, items, count, ws);
  else
    hipLaunchKernelGGL(wq_pack_kernel<float>, dim3(256, count), dim3(256), 0, st, items, count, ws);
  return rn_check_launch("weight_quant_pack");
}

int rn_quant_int8_bwd(int32_t dtype, int64_t n, const void* x, const void* dy, void* dx, const float* minmax,
                      int32_t is_weight, const void* add_src, rn_stream_t stream) {
  RN_CHECK_ARG(x && dy && dx && n > 0, "bad arguments");
  hipStream_t st = as_stream(stream);
  if (dtype == RN_BF16)
    hipLaunchKernelGGL(quant_bwd_kernel<bf16_t>, dim3(grid1d(n)), dim3(256), 0, st, n, (const bf16_t*)x,
                       (const bf16_t*)dy, (bf16_t*)dx, minmax, is_weight, (const bf16_t*)add_src);
  else
    hipLaunchKernelGGL(quant_bwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st, n, (const float*)x,
                       (const float*)dy, (float*)dx, minmax, is_weight, (const float*)add_src);
  return rn_check_launch("quant_int8_bwd");
}

}  // extern "C"
