// rn_conv.hip -- Convolution / FullyConnected on CDNA4 MFMA (gfx950).
//
// Replaces the cuDNN conv fwd / bwd-data / bwd-filter that MXNet ran for mx.sym.Convolution
// (reference symbol/resnet.py:14-31,93, symbol/resnext.py:17-38,83) and the cuBLAS GEMM of
// mx.sym.FullyConnected (symbol/resnet.py:115). Activations are NHWC, weights KRSC.
//
//  * igemm_kernel   : y[M=N*P*Q][K] = gather(x)[M][R*S*C] * W^T, the implicit GEMM used for
//                     forward AND for data-gradient (a transposed conv, split into stride
//                     parity classes so that only valid taps are visited).
//  * wgrad_kernel   : dW[K][R*S*C] += dy^T[K][M] * gather(x)[M][R*S*C], split over M with
//                     fp32 atomics; both operands are read from LDS with ds_read_b64_tr_b16.
//  * im2col / pack / stem-shift-grad helpers.
//
// Tile anatomy (igemm): 256 threads = 4 waves in 2x2, block tile BM x BN, one K stage is
// 128 bytes of reduction per row (64 bf16 / 32 f32), register-staged global->LDS with the
// write placed after the MFMA phase (async-STAGE split), LDS double buffered, one barrier
// per stage, 16-byte chunks XOR-swizzled by (row & 7) so ds_read_b128 fragment reads are
// bank-conflict free.  bf16: v_mfma_f32_16x16x32_bf16.  f32: v_mfma_f32_16x16x4_f32 (exact
// fp32 products, used by the parity path).
#include "rn_common.h"

namespace {

// CUs of the device (cached once per process; 256 -- gfx950 MI355X -- on a host without a GPU, where
// only plan-time sizing runs): the split-M weight gradients size their grids to one round of it
int chip_cus() {
  static const int cus = [] {
    const int n = rn_device_cu_count();
    return n > 0 ? n : 256;
  }();
  return cus;
}
// CUs the weight gradients size their split-M grids for: the chip, scaled by rn_set_tuning 21 (percent,
// default 50; 0 = 100). They share the chip with the data-gradient chain on the other stream: half the
// splits halve the partial slabs written and reduced, and the data gradients keep more of the CUs
// (ResNet-50: 100 % 20.83, 50 % 20.09 ms per step; 45 % 0.8 % below 50 with HIP events in every step, 1.2 %
// above it without them, round 6; a quarter starves the weight
// gradients: 23.85)
int wgrad_cus() {
  const int pct = g_tune[RN_TUNE_WGRAD_SPLIT] > 0 ? g_tune[RN_TUNE_WGRAD_SPLIT] : 100;
  return std::max(8, chip_cus() * pct / 100);
}

// ------------------------------------------------------------------------------ igemm
struct IgemmCls {
  int a, b;          // output parity class (dgrad) -- (0,0) for fwd
  int Pc, Qc;        // class-local output extent
  int r0, s0;        // first tap of the class
  int nr, ns;        // taps in the class
  int hoff0, woff0;  // gathered coordinate offset of tap 0
  int hb0, wb0;      // row-coordinate bias
  FastDiv fdQ, fdPQ;
};

struct IgemmArgs {
  const void* x;
  const void* w;
  void* y;
  const void* add;
  const float* bias;
  int N, H, W, C;      // gathered tensor; C = channel stride (multiple of the chunk)
  int P, Q;            // output tensor spatial
  int K, ldo;          // valid output columns, output row stride
  int S;               // taps per weight row (for the B row offset)
  int wrow;            // B matrix row stride = R*S*C
  int rstep, sstep;    // tap step (1 fwd, stride dgrad)
  int hmul, wmul;      // row coordinate multiplier (stride fwd, 1 dgrad)
  int hinc, winc;      // gathered coordinate change per tap step (+1 fwd, -1 dgrad)
  int ostep_h, ostep_w;
  int gcol, gred;      // grouped: output columns / reduction channels per group (dense: 2^30, 0)
  int cblk;            // reduction channels per column block (dense: C)
  float* stats;        // fwd only, nullable: per-block BatchNorm partials [m tiles][3][ldo]
  float* stats_mm;     // fwd (EPI 1) only, nullable: per-block extreme of the stored output [m tiles][ldo]:
  const float* mm_sign;  // the max, or the min where mm_sign[col] < 0 (nullable: the max everywhere)
  const float* in_sc;  // fwd only, nullable: BN+ReLU applied to the gathered input while staging
  const float* in_sh;
  int ntn;             // n tiles (grid = m tiles * ntn)
  int smallc, lgc, rs; // fwd over C < one stage (the stem's 8 channels): k = tap*C + c flattened
  int diag_l1;         // diagnostic (rn_set_tuning 3): every A row reads the same L1-resident chunk
  int sched;           // igemm_big_kernel schedule experiments (rn_set_tuning 7, bit mask)
  int epi_sync;        // igemm_big_kernel: block barriers around the epilogue's LDS staging (rn_set_tuning 16)
  int nt_store;        // igemm_big_kernel: output stores with the nontemporal hint (rn_set_tuning 18 bit 16)
  int prio;            // igemm_big_kernel 8-wave tiles: waves 4-7 at s_setprio 1 for the whole kernel (rn_set_tuning 20)
  int ntiles;          // igemm_big_kernel persistent mode: tiles per class (0: one tile per workgroup)
  int x_bytes, w_bytes;  // LDS-DMA buffer descriptors
  // dgrad only, nullable: the BatchNorm-backward reduction of the gradient this conv completes
  // (sum dz, sum dz*(x - mean), dz = dy * relu'(bn(x))) per output block -> bnred[blk][ldo][2]
  float* bnred;
  const void* bn_x;
  const float *bn_mean, *bn_sc, *bn_sh;
  int bn_relu, mt_max;
  // dgrad only, nullable (igemm_big_kernel EPI 3): the BatchNorm backward APPLIED to the recomputed
  // gradient g (rounded as stored): dx = A (dz - mean dz) - A2 (x - mean) (+ add), coefficients
  // {A, mean dz, A2, mean} per channel from rn_bn_bwd_finalize, x = bn_x, dz = g relu'(x sc + sh)
  const float* bn_coef;
  // dgrad only, nullable: a folded Quantization_int8 straight-through clip on the BN output (rn_bn_desc.clip)
  const float* bn_clip;
  const float* bn_clip2;  // (EPI 4) nullable: a quantizer pair -- add is the other quantizer's gradient (below)
  // int8 forward (igemm_big_kernel Q8): per-tensor quantization units of the int8 codes in x and w
  // (Quantization_int8: value = code * unit); the int32 accumulators are scaled by their product
  const float* qunit_x;
  const float* qunit_w;
  FastDiv fdS;
  int ncls;
  int ksplit;          // igemm_kernel, fp32 output, one-tap 1x1 reductions: split-K over blockIdx.y, fp32
                       // atomic adds into the zeroed output (the FC forward's 16-tile grids)
  IgemmCls cls[4];
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }
// swizzle for 32x32x16 fragment reads (32 lanes read 32 consecutive rows at one chunk): the
// 16-lane ds_read_b128 groups {0-3,12-15,20-27} / {4-11,16-19,28-31} then cover 16 distinct
// 16-byte slots of a 256-byte line pair (row & 15 distinct within each group)
__device__ __forceinline__ int swz32(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef float v16f __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void mfma32(v16f& acc, const uint4& a, const uint4& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8s, a), __builtin_bit_cast(v8s, b), acc, 0, 0, 0);
}

// LDS-DMA (buffer_load ... lds) of one 16-byte chunk per lane: the LDS destination is the
// wave-uniform base + 16 * lane; an out-of-range voffset reads zeros (halo / ragged edges).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, const void* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff,
                                           0, 0, 0);
}
constexpr uint32_t kOob = 0xFFFFFFF0u;
// channels of the BatchNorm+ReLU input transform the LDS-DMA kernels keep in LDS (XF; W4 tile)
constexpr int kXfMaxC = 2048, kXfMaxCW4 = 512;

// XCD-aware block order: the dispatcher deals consecutive workgroup ids round-robin over the 8
// XCDs (each with a private L2). Bijective remap so that every XCD walks a contiguous range of
// logical tiles: neighbouring tiles (which share operand panels) then share an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <typename T>
__device__ __forceinline__ void mfma_slab(v4f& acc, const uint4& a, const uint4& b);

template <>
__device__ __forceinline__ void mfma_slab<bf16_t>(v4f& acc, const uint4& a, const uint4& b) {
  v8s av = __builtin_bit_cast(v8s, a);
  v8s bv = __builtin_bit_cast(v8s, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma_slab<float>(v4f& acc, const uint4& a, const uint4& b) {
  // lane group g holds k = 4g..4g+3; MFMA step e pairs A[.][4g+e] with B[4g+e][.]
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}

template <typename OutT>
__device__ __forceinline__ float load_out(const void* p, int64_t i) {
  return to_f(reinterpret_cast<const OutT*>(p)[i]);
}

// BatchNorm statistics of the block's output rows, from the staged (stored-precision) fp32 tile:
// per column, pivot p = row 0's value, S1 = sum(v - p), S2 = sum((v - p)^2) over the block's
// valid rows -> part[blk][0|1|2][col] (merged exactly in fp64 by rn_bn_fwd_train_part).
template <int BM, int BN, int LDT>
__device__ __forceinline__ void bn_stats_epilogue(float* tile, float* __restrict__ part, int ld, int m0, int n0,
                                                  int Mc, int mtile) {
  constexpr int TPC = 256 / BN;  // threads per column
  const int tid = threadIdx.x;
  const int col = tid % BN, sub = tid / BN;
  const int nv = min(BM, Mc - m0);
  __syncthreads();
  const float piv = tile[col];
  float s1 = 0.f, s2 = 0.f;
  for (int r = sub; r < nv; r += TPC) {
    const float d = tile[r * LDT + col] - piv;
    s1 += d;
    s2 = fmaf(d, d, s2);
  }
  __syncthreads();
  tile[(2 * sub) * LDT + col] = s1;
  tile[(2 * sub + 1) * LDT + col] = s2;
  __syncthreads();
  if (sub == 0 && n0 + col < ld) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int t = 0; t < TPC; ++t) {
      a += tile[(2 * t) * LDT + col];
      b += tile[(2 * t + 1) * LDT + col];
    }
    float* dst = part + (int64_t)mtile * 3 * ld + n0 + col;
    dst[0] = a;
    dst[ld] = b;
    dst[2 * ld] = piv;
  }
}

template <typename T, typename OutT, int BM, int BN, bool DMA = false>
__global__ __launch_bounds__(256, 2) void igemm_kernel(IgemmArgs p) {
  constexpr int CE = 16 / sizeof(T);   // elements per chunk
  constexpr int BKE = 128 / sizeof(T); // reduction elements per stage
  constexpr int A_CH = BM / 32;        // chunks per thread per stage (A)
  constexpr int B_CH = BN / 32;
  constexpr int MI = BM / 32;          // 16x16 tiles per wave (rows)
  constexpr int NI = BN / 32;
  // one LDS arena: double-buffered A/B stages in the K loop, the fp32 output tile after it
  constexpr int kStageChunks = 2 * (BM + BN) * 8;
  constexpr int kTileChunks = BM * (BN + 4) * 4 / 16;
  __shared__ __attribute__((aligned(16))) uint4 smem[kStageChunks > kTileChunks ? kStageChunks : kTileChunks];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const IgemmCls& cl = p.cls[blockIdx.z];
  const int Mc = p.N * cl.Pc * cl.Qc;
  // 1-D grid over (m tile, n tile), n fastest: the n tiles reading one gathered A panel are
  // consecutive logical blocks and, after the remap, run on one XCD
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int mtile = lid / p.ntn;
  const int m0 = mtile * BM;
  const int n0 = (lid - mtile * p.ntn) * BN;
  if (m0 >= Mc) {  // (a dgrad parity class with fewer rows): empty BN-reduction partials
    if (p.bnred)
      for (int col = threadIdx.x; col < BN; col += 256)
        if (n0 + col < p.ldo) {
          float* dst = p.bnred + ((int64_t)(blockIdx.z * p.mt_max + mtile) * p.ldo + n0 + col) * 2;
          dst[0] = 0.f;
          dst[1] = 0.f;
        }
    return;
  }
  // grouped conv: the block's columns touch groups n0/gcol.., whose input channels start here
  const int cbase = (n0 / p.gcol) * p.gred;

  const T* __restrict__ xg = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ wg = reinterpret_cast<const T*>(p.w);

  // ---- per-thread load assignment: chunk column ch, rows (tid>>3) + 32*i
  const int ch = tid & 7;
  int a_pix[A_CH];  // n*H*W
  int a_hb[A_CH], a_wb[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    if (m < Mc) {
      const int n = fdiv(m, cl.fdPQ);
      const int rem = m - n * cl.Pc * cl.Qc;
      const int ii = fdiv(rem, cl.fdQ);
      const int jj = rem - ii * cl.Qc;
      a_pix[i] = n * p.H * p.W;
      a_hb[i] = ii * p.hmul + cl.hb0;
      a_wb[i] = jj * p.wmul + cl.wb0;
    } else {
      a_pix[i] = 0;
      a_hb[i] = -(1 << 28);  // never in range
      a_wb[i] = 0;
    }
  }
  // LDS-DMA staging writes each wave's 1 KiB lane-linearly (lane l -> row 8w + l/8 (+32 i), slot
  // l&7), so a lane fetches the source chunk the XOR read-swizzle expects in that slot; the XOR
  // term (row & 7) is the same for all of a thread's rows.
  const int lch = DMA ? (ch ^ ((tid >> 3) & 7)) : ch;
  // DMA fast path: per row, the gathered offset of tap (0,0) and a bitmask of the class's taps that
  // land inside the image, so a stage costs one shift/and/add/select per row
  int a_row[DMA ? A_CH : 1];
  uint64_t a_mask[DMA ? A_CH : 1];
  if constexpr (DMA) {
    if (!p.smallc) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        uint64_t msk = 0;
        for (int tr = 0; tr < cl.nr; ++tr) {
          const int hin = a_hb[i] + cl.hoff0 + p.hinc * tr;
          if ((unsigned)hin >= (unsigned)p.H) continue;
          for (int ts = 0; ts < cl.ns; ++ts) {
            const int win = a_wb[i] + cl.woff0 + p.winc * ts;
            if ((unsigned)win < (unsigned)p.W) msk |= 1ull << (tr * cl.ns + ts);
          }
        }
        a_mask[i] = msk;
        a_row[i] = msk ? (a_pix[i] + (a_hb[i] + cl.hoff0) * p.W + a_wb[i] + cl.woff0) * p.C + cbase + lch * CE : 0;
      }
    }
  }
  int b_off[B_CH];  // 32-bit: weight matrices are far below 2^31 elements (host-checked)
  bool b_ok[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int col = n0 + (tid >> 3) + 32 * i;
    b_ok[i] = col < p.K;
    b_off[i] = (b_ok[i] ? col : 0) * p.wrow;
  }

  const int ncb = (p.cblk + BKE - 1) / BKE;
  int nstage = p.smallc ? (p.rs * p.C + BKE - 1) / BKE : cl.nr * cl.ns * ncb;
  int kbeg = 0;  // split-K (host: one tap, no smallc): this split's channel-block range
  if (p.ksplit > 1) {
    const int per = (nstage + p.ksplit - 1) / p.ksplit;
    kbeg = blockIdx.y * per;
    nstage = max(0, min(nstage, kbeg + per) - kbeg);
  }

  // register-staged loads: stage t+1 is loaded while stage t is computed, then written to
  // the other LDS buffer (async-STAGE split: write after the MFMA phase).
  uint4 ra0[A_CH], rb0[B_CH];
  int st_tr = 0, st_ts = 0, st_cb = kbeg;  // next stage to load
  int st_buf = 0;                       // LDS buffer the next DMA stage lands in
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.w_bytes, 0x00020000);

  // BN+ReLU input transform (in_sc): the stage's channel coefficients are loaded with its chunks and
  // applied when the chunks are written to LDS (store_stage, after the MFMA phase), so the loads stay
  // in flight under the MFMAs; chunks outside the image stay zero (the conv pads the BN+ReLU output)
  float xsc[CE], xsh[CE];
  uint32_t xok = 0;
  auto load_stage = [&](uint4* ra, uint4* rb) {
    int hoff, woff, c, toff;
    int dtr = 0, dts = 0, dcb = 0;  // stage's tap / channel-block (DMA fast path)
    bool cok;
    if (p.smallc) {
      // several taps per stage: this thread's chunk is k = tap*C + c of the flattened reduction
      const int k0 = st_cb * BKE + lch * CE;
      ++st_cb;
      const int tap = k0 >> p.lgc;
      c = k0 & (p.C - 1);
      hoff = (int)fdiv((uint32_t)tap, p.fdS);
      woff = tap - hoff * p.S;
      cok = tap < p.rs;
      toff = k0;
    } else {
      const int tr = st_tr, ts = st_ts, cb = st_cb;
      dtr = tr; dts = ts; dcb = cb;
      if (++st_cb == ncb) {
        st_cb = 0;
        if (++st_ts == cl.ns) {
          st_ts = 0;
          ++st_tr;
        }
      }
      const int r = cl.r0 + p.rstep * tr;
      const int s = cl.s0 + p.sstep * ts;
      hoff = cl.hoff0 + p.hinc * tr;
      woff = cl.woff0 + p.winc * ts;
      c = cb * BKE + lch * CE;
      cok = c < p.cblk && cbase + c < p.C;  // a grouped block may run past the last group
      toff = (r * p.S + s) * p.cblk + c;
    }
    if constexpr (DMA) {
      const int buf = st_buf;
      st_buf ^= 1;
      const uint4* As = smem + buf * (BM + BN) * 8;
      const uint4* Bs = As + BM * 8;
      const int wrow = (tid >> 6) * 8;  // first row of this wave's 1 KiB piece
      if (!p.smallc) {
        // uniform per stage: tap index inside the class and its offset from tap (0,0)
        const int tapi = dtr * cl.ns + dts;
        const int toffa = ((hoff - cl.hoff0) * p.W + (woff - cl.woff0)) * p.C + dcb * BKE;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
          const bool ok = cok && ((a_mask[i] >> tapi) & 1ull);
          const uint32_t off = ok ? (uint32_t)((a_row[i] + toffa) * (int)sizeof(T)) : kOob;
          dma16(rs_x, As + (wrow + 32 * i) * 8, off);
        }
      } else {
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
          const int hin = a_hb[i] + hoff;
          const int win = a_wb[i] + woff;
          const bool ok = cok && (unsigned)hin < (unsigned)p.H && (unsigned)win < (unsigned)p.W;
          const uint32_t off =
              ok ? (uint32_t)(((a_pix[i] + hin * p.W + win) * p.C + cbase + c) * (int)sizeof(T)) : kOob;
          dma16(rs_x, As + (wrow + 32 * i) * 8, off);
        }
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const uint32_t off = (cok && b_ok[i]) ? (uint32_t)((b_off[i] + toff) * (int)sizeof(T)) : kOob;
        dma16(rs_w, Bs + (wrow + 32 * i) * 8, off);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int hin = a_hb[i] + hoff;
      const int win = a_wb[i] + woff;
      const bool ok = cok && (unsigned)hin < (unsigned)p.H && (unsigned)win < (unsigned)p.W;
      if (ok) {
        const int off = (kRnDiag && p.diag_l1) ? (c & 63) : (a_pix[i] + hin * p.W + win) * p.C + cbase + c;  // < 2^31
        ra[i] = *reinterpret_cast<const uint4*>(xg + off);
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
      if (i == 0) xok = 0;
      xok |= (uint32_t)ok << i;
    }
    if (p.in_sc && cok) {
#pragma unroll
      for (int e = 0; e < CE; e += 4) {
        *reinterpret_cast<float4*>(xsc + e) = *reinterpret_cast<const float4*>(p.in_sc + cbase + c + e);
        *reinterpret_cast<float4*>(xsh + e) = *reinterpret_cast<const float4*>(p.in_sh + cbase + c + e);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      if (cok && b_ok[i]) rb[i] = *reinterpret_cast<const uint4*>(wg + b_off[i] + toff);
      else rb[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_stage = [&](int buf, const uint4* ra, const uint4* rb) {
    uint4* As = smem + buf * (BM + BN) * 8;
    uint4* Bs = As + BM * 8;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = (tid >> 3) + 32 * i;
      uint4 v = ra[i];
      if (p.in_sc) {
        float f[CE];
        chunk_to_f(v, f, (const T*)nullptr);
#pragma unroll
        for (int e = 0; e < CE; ++e) f[e] = fmaxf(fmaf(f[e], xsc[e], xsh[e]), 0.f);
        v = ((xok >> i) & 1u) ? f_to_chunk(f, (const T*)nullptr) : make_uint4(0, 0, 0, 0);
      }
      As[row * 8 + swz(row, ch)] = v;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = (tid >> 3) + 32 * i;
      Bs[row * 8 + swz(row, ch)] = rb[i];
    }
  };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint4* As = smem + buf * (BM + BN) * 8;
    const uint4* Bs = As + BM * 8;
#pragma unroll
    for (int slab = 0; slab < 2; ++slab) {
      uint4 af[MI], bfr[NI];
      const int kc = slab * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * (BM / 2) + i * 16 + (lane & 15);
        af[i] = As[row * 8 + swz(row, kc)];
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wn * (BN / 2) + j * 16 + (lane & 15);
        bfr[j] = Bs[row * 8 + swz(row, kc)];
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) mfma_slab<T>(acc[i][j], af[i], bfr[j]);
    }
  };

  // ---- epilogue chunk assignment (decoded once; residual chunks prefetched in the last stage)
  constexpr int OE = 16 / sizeof(OutT);  // output elements per 16-byte chunk
  constexpr int CPR = BN / OE;           // chunks per tile row
  constexpr int EPC = BM * CPR / 256;    // epilogue chunks per thread
  constexpr int EPH = EPC >= 2 ? EPC / 2 : 1;  // processed in halves (register pressure)
  const OutT* __restrict__ ag = reinterpret_cast<const OutT*>(p.add);
  int64_t ep_off[EPH];
  uint4 ep_add[EPH];
  uint4 ep_x[EPH];
  const T* __restrict__ bxg = reinterpret_cast<const T*>(p.bn_x);
  auto prefetch_add = [&](int half) {
#pragma unroll
    for (int k = 0; k < EPH; ++k) {
      const int cidx = tid + 256 * (k + half * EPH);
      const int row = cidx / CPR;
      const int cc = cidx - row * CPR;
      const int m = m0 + row;
      const int col0 = n0 + cc * OE;
      ep_off[k] = -1;
      ep_add[k] = make_uint4(0, 0, 0, 0);
      if (m < Mc && col0 < p.K) {
        const int n = fdiv(m, cl.fdPQ);
        const int rem = m - n * cl.Pc * cl.Qc;
        const int ii = fdiv(rem, cl.fdQ);
        const int jj = rem - ii * cl.Qc;
        const int oh = cl.a + p.ostep_h * ii;
        const int ow = cl.b + p.ostep_w * jj;
        ep_off[k] = ((int64_t)(n * p.P + oh) * p.Q + ow) * p.ldo + col0;
        if (ag && col0 + OE <= p.K) ep_add[k] = *reinterpret_cast<const uint4*>(ag + ep_off[k]);
        if (p.bnred) ep_x[k] = *reinterpret_cast<const uint4*>(bxg + ep_off[k]);
      }
    }
  };

  if constexpr (DMA) {
    // LDS-DMA: no staging registers and no ds_write pass (the VGPR->LDS store path is the slowest
    // LDS path); stage t+1 is in flight while stage t is computed
    if (nstage > 0) {
      load_stage(ra0, rb0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    for (int t = 0; t < nstage; ++t) {
      if (t + 1 < nstage) load_stage(ra0, rb0);
      compute(t & 1);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
  } else {
    if (nstage > 0) {
      load_stage(ra0, rb0);
      store_stage(0, ra0, rb0);
      __syncthreads();
    }
    for (int t = 0; t < nstage; ++t) {
      const bool more = t + 1 < nstage;
      if (more) load_stage(ra0, rb0);
      compute(t & 1);
      if (more) store_stage((t + 1) & 1, ra0, rb0);
      __syncthreads();
    }
  }

  // ---- epilogue: stage the fp32 tile through LDS, then every thread writes whole 16-byte
  // output chunks along a row (+bias, +prefetched add_src chunk).
  constexpr int LDT = BN + 4;  // fp32 row stride of the staged tile (pad: 2-way -> conflict-free)
  static_assert(BM * LDT * 4 <= (int)sizeof(smem), "epilogue tile does not fit the staging LDS");
  static_assert(BM * CPR % 256 == 0, "epilogue chunks must divide over the block");
  float* tile = reinterpret_cast<float*>(smem);
  prefetch_add(0);  // residual loads fly while the accumulator tile is staged
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + e;
        const int col = wn * (BN / 2) + j * 16 + (lane & 15);
        tile[row * LDT + col] = acc[i][j][e];
      }
  __syncthreads();
  OutT* __restrict__ yg = reinterpret_cast<OutT*>(p.y);
  // BN-backward reduction: this thread's column chunk is fixed (256 % CPR == 0)
  float r_mu[OE], r_sc[OE], r_sh[OE], r1[OE], r2[OE];
  if (p.bnred) {
    const int c0 = n0 + (tid % CPR) * OE;
#pragma unroll
    for (int e = 0; e < OE; ++e) {
      const bool okc = c0 + e < p.K;
      r_mu[e] = okc ? p.bn_mean[c0 + e] : 0.f;
      r_sc[e] = okc ? p.bn_sc[c0 + e] : 0.f;
      r_sh[e] = okc ? p.bn_sh[c0 + e] : 0.f;
      r1[e] = r2[e] = 0.f;
    }
  }
#pragma unroll
  for (int half = 0; half < EPC / EPH; ++half) {
  if (half > 0) prefetch_add(half);
#pragma unroll
  for (int k = 0; k < EPH; ++k) {
    if (ep_off[k] < 0) continue;
    const int cidx = tid + 256 * (k + half * EPH);
    const int row = cidx / CPR;
    const int cc = cidx - row * CPR;
    const int col0 = n0 + cc * OE;
    float v[OE];
#pragma unroll
    for (int e = 0; e < OE; ++e) v[e] = tile[row * LDT + cc * OE + e];
    if (p.bias && blockIdx.y == 0) {
#pragma unroll
      for (int e = 0; e < OE; ++e) v[e] += (col0 + e < p.K) ? p.bias[col0 + e] : 0.f;
    }
    if constexpr (std::is_same<OutT, float>::value) {
      if (p.ksplit > 1) {  // split-K: partial sums added into the zeroed fp32 output
        for (int e = 0; e < OE && col0 + e < p.K; ++e) atomicAdd(yg + ep_off[k] + e, v[e]);
        continue;
      }
    }
    if (col0 + OE <= p.K) {  // full chunk: vector path
      if (ag) {
        float a[OE];
        chunk_to_f(ep_add[k], a, (const OutT*)nullptr);
#pragma unroll
        for (int e = 0; e < OE; ++e) v[e] += a[e];
      }
      const uint4 out = f_to_chunk(v, (const OutT*)nullptr);
      *reinterpret_cast<uint4*>(yg + ep_off[k]) = out;
      if (p.bnred) {  // on the stored (rounded) gradient, as a separate BN-backward pass would read it
        float g[OE], xv[OE];
        chunk_to_f(out, g, (const OutT*)nullptr);
        chunk_to_f(ep_x[k], xv, (const T*)nullptr);
#pragma unroll
        for (int e = 0; e < OE; ++e) {
          const float dz = (!p.bn_relu || fmaf(xv[e], r_sc[e], r_sh[e]) > 0.f) ? g[e] : 0.f;
          r1[e] += dz;
          r2[e] = fmaf(dz, xv[e] - r_mu[e], r2[e]);
        }
      }
      if (p.stats) {  // keep the stored (rounded) values for the BatchNorm statistics below
        chunk_to_f(out, v, (const OutT*)nullptr);
#pragma unroll
        for (int e = 0; e < OE; ++e) tile[row * LDT + cc * OE + e] = v[e];
      }
    } else {  // ragged last chunk (num_hidden % 8 != 0)
      for (int e = 0; e < OE && col0 + e < p.K; ++e) {
        float o = v[e];
        if (ag) o += to_f(ag[ep_off[k] + e]);
        yg[ep_off[k] + e] = from_f<OutT>(o);
      }
    }
  }
  }
  if (p.stats) bn_stats_epilogue<BM, BN, LDT>(tile, p.stats, p.ldo, m0, n0, Mc, mtile);
  if (p.bnred) {
    // rows -> one partial per column: lanes sharing the column chunk (stride CPR) first, then waves
#pragma unroll
    for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
      for (int e = 0; e < OE; ++e) {
        r1[e] += __shfl_xor(r1[e], off, 64);
        r2[e] += __shfl_xor(r2[e], off, 64);
      }
    __syncthreads();  // the staged tile is no longer read
    float* red = tile;  // [wave][CPR][OE][2]
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < OE; ++e) {
        red[((wid * CPR + lane) * OE + e) * 2] = r1[e];
        red[((wid * CPR + lane) * OE + e) * 2 + 1] = r2[e];
      }
    }
    __syncthreads();
    if (tid < CPR * OE) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        a += red[((w * CPR) * OE + tid) * 2];
        b += red[((w * CPR) * OE + tid) * 2 + 1];
      }
      if (n0 + tid < p.ldo) {
        float* dst = p.bnred + ((int64_t)(blockIdx.z * p.mt_max + mtile) * p.ldo + n0 + tid) * 2;
        dst[0] = a;
        dst[1] = b;
      }
    }
  }
}

// ------------------------------------------------------------------------------ igemm, 256-row tiles
// The same implicit GEMM (fwd and dgrad classes, bf16 in / bf16 out, optional residual add) on a
// 256 x BN tile run by 8 waves (2 along M x 4 along N, each 128 x BN/4): twice the MFMA work per
// staged byte of the 128 x 128 kernel, one workgroup per CU. Both operands are staged by LDS-DMA
// (buffer_load ... lds, 16 B per lane; padding / halo rows read zeros through an out-of-range
// offset) issued from inline asm, so hipcc does not drain them before every ds_read: NBUF K-tile
// buffers, NBUF-1 K-tiles in flight, one counted vmcnt + barrier per 64-deep K-tile. The epilogue
// stages each wave's accumulators through LDS in two 64-row halves and writes 16-byte row chunks.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v4i make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  v4i r;  // readfirstlane: provably wave-uniform, so the asm "s" operand gets SGPRs
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xFFFFu));  // stride 0
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// one 16-byte LDS-DMA per lane into the wave-uniform LDS byte address lds (+16 * lane); M0 is
// compiler-reserved, so it is saved and restored inside the statement. No "memory" clobber: the
// LDS it writes is ordered by the explicit wait_vmcnt + barrier (which carry one), and without it
// the compiler keeps kernel arguments in SGPRs and schedules the fragment reads across the DMAs.
__device__ __forceinline__ void dma16_asm(const v4i& rsrc, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  lds = __builtin_amdgcn_readfirstlane(lds);  // free when already scalar; M0 is written by an SALU move
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(rsrc));
}

// the same through global_load_lds_dwordx4 with a per-lane 64-bit source address (no buffer
// descriptor in SGPRs); masked lanes read a zero chunk
__device__ __attribute__((aligned(16))) const uint4 g_zero_chunk = {0u, 0u, 0u, 0u};

__device__ __forceinline__ void dma16_global(const void* src, uint32_t lds) {
  uint32_t keep;
  lds = __builtin_amdgcn_readfirstlane(lds);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// EPI: 0 plain; 1 (fwd) BatchNorm statistics of the stored output per 128-row half (one wave row):
// part[2*mtile + wm][S1 | S2 | pivot][ldo], as igemm_kernel's bn_stats_epilogue; 2 (dgrad) the
// BatchNorm-backward reduction of the stored gradient: bnred[class][2*mtile + wm][ldo][2].
// BN = 64 (the 64-channel layers): 4 waves stacked along M (each 64 x 64), two workgroups per CU;
// plain epilogue only (EPI 0).
// M32: v_mfma_f32_32x32x16_bf16 (32-cycle MFMAs: three times the issue shadow of the 16x16x32
// form for the fragment reads, DMA address arithmetic and waits of the same K-tile) with the
// swz32 LDS image; else v_mfma_f32_16x16x32_bf16 with swz.
// BM: tile rows, 256 or 224 (16x16 MFMAs only: 112 rows per wave row). M = N*P*Q is 256 * 49 * 4^j
// for every ResNet-50 layer at batch 256, so 256-row tiles leave a last round of 196 / 256 workgroups
// on every grid; 224-row tiles (7 / 8 of the rows) fill 224 / 256. The A region of the LDS stage
// keeps 256 rows (the DMA rounds of rows >= BM read zeros).
// Q8: int8 operands (the int8 codes of Quantization_int8, symbol/int8_api.py:120-171), 128-deep
// K-tiles of the same 128-byte rows, v_mfma_i32_16x16x64_i8 (exact int32 sums; the A and B fragments
// take the same 16-byte chunks as the bf16 form, so the LDS images and reads are unchanged), the
// accumulators scaled by unit_x * unit_w in the epilogue; output bf16 (Q8 1) or fp32 (Q8 2).
// SC: the stem's small-C modes (64-column tile only), where a DMA lane's chunk of a K-tile is its own
// tap, so the gathered row offset (and the in-image test) is per lane. SC 1: NHWC with C = 8 (one
// tap per 16-byte chunk, k = tap * 8 + c). SC 2: the padded NHWC4 image of rn_stem_prepare_p4 (zero
// border, so no in-image test): k = (r * 8 + s) * 4 + c over r, s < 8 (tap 7 of a row and row 7
// have zero weights), a chunk = taps (r, 2 j) and (r, 2 j + 1), K-tile t = rows 2 t, 2 t + 1.
// XF: the producing BatchNorm+ReLU applied on load (forward of the pre-activation units' convs,
// symbol/resnet.py:17-31: act = relu(bn(x)) is never written). in_sc / in_sh (<= kXfMaxC channels)
// are copied into LDS once; each thread rewrites its own landed A chunks in place, max(x*sc + sh, 0)
// rounded to bf16 exactly as bn_apply_kernel does, between the K-tile's vmcnt wait and its barrier.
// Chunks the DMA zero-filled (halo taps, rows past the tile) stay zero: the conv pads the BN+ReLU
// output with zeros.
// W4: the 224x128 tile on 4 waves (2 x 2, each 112 x 64, the wave tile of the 224x256 kernel) with
// ONE K-tile buffer: 72 KB of LDS, two workgroups per CU, so one workgroup's epilogue (its output
// stores and LDS staging) overlaps the other's loads and MFMAs. For 1x1, pad-0 convolutions with at
// most two K-tiles (their tiles are load / store bound: the 8-wave tiles alternate a read+MFMA phase
// and a write phase on each CU); no halo, so the DMA rows need no in-image test.
// GD: grouped convolutions with as many output columns as input channels per group (ResNeXt's 3x3,
// symbol/resnext.py:23-25), <= 32 per group, on the 64-column tile: block column c and block channel c
// belong to the same group, so an MFMA of k-step ks and column sub-block j multiplies zeros unless the
// channel range of ks lies in the column range of j (32x32x16: ks >> 1 == j; 16x16x32: j >> 1 == ks).
// Those MFMAs and their B-fragment reads are skipped: half the MFMA work of the block-diagonal tile.
// EPIX 4: EPI 2 whose BatchNorm output feeds a Quantization_int8 (rn_conv_bwd_data_bnred_clip): dz also
// carries the quantizer's straight-through clip (a compile-time variant: the other epilogues keep
// their code)
template <int BN, int NBUF, int EPIX = 0, bool M32 = false, int BM = 256, int SC = 0, int Q8 = 0, int XF = 0, int W4 = 0,
          int GD = 0>
__global__ __launch_bounds__(BN == 64 || W4 ? 256 : 512, BN == 64 || W4 ? 2 : 1) void igemm_big_kernel(IgemmArgs p) {
  constexpr int EPI = EPIX == 4 ? 2 : EPIX == 5 ? 1 : EPIX;
  constexpr bool CLIP = EPIX == 4;
  constexpr bool MM = EPIX == 5;  // EPI 1 + the per-block extremes of the stored output (p.stats_mm)
  constexpr int ES = Q8 ? 1 : 2;                 // operand bytes per element
  constexpr int BMA = 256, CE = 16 / ES, BKE = 128 / ES;
  using OutT = typename std::conditional<Q8 == 2, float, bf16_t>::type;
  constexpr int NW = BN == 64 || W4 ? 4 : 8;     // waves
  constexpr int WAVES_N = BN == 64 ? 1 : W4 ? 2 : 4, WAVES_M = NW / WAVES_N;
  static_assert(!W4 || (BN == 128 && BM == 224 && NBUF == 1 && !M32 && !SC && !Q8), "W4 tile");
  constexpr int XFC = W4 ? kXfMaxCW4 : kXfMaxC;   // (XF) channels of the LDS scale / shift table
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;  // wave tile
  constexpr int RPR = NW * 8;                    // rows per DMA round (8 per wave)
  constexpr int AR = BMA / RPR, BR = BN / RPR;   // DMA rounds per K-tile
  constexpr int LPT = AR + BR;                   // DMA instructions per thread per K-tile
  constexpr int FM = M32 ? 32 : 16;              // MFMA tile edge
  constexpr int MI = WM / FM, NI = WN / FM;      // accumulators per wave
  constexpr int NCH = (WM + 63) / 64;            // 64-row epilogue chunks per wave
  // BatchNorm partials (EPI 1 / 2): the two wave rows of the 8-wave and W4 tiles share one partial
  // per tile (one pivot, sums combined through LDS), halving what the merge / finalize passes read;
  // the 64-column tile keeps one per 64-row wave row
  constexpr bool PAIR = WAVES_M == 2;
  constexpr int PR = PAIR ? 1 : WAVES_M;         // BatchNorm partials per tile
  static_assert(WM % FM == 0 && (BM == 256 || !M32) && (BM == 256 || BN != 64) && (!SC || BN == 64), "tile shape");
  static_assert(!Q8 || (!M32 && !SC && EPI != 2), "int8: 16x16x64 MFMAs, forward only");
  using AccT = typename std::conditional<Q8 != 0, v4i, typename std::conditional<M32, v16f, v4f>::type>::type;
  constexpr int kStage = (BMA + BN) * 8;         // 16-byte chunks per K-tile
  constexpr int EP_LD = WN + 4;                  // staged fp32 row stride
  constexpr int EP_WAVE = 64 * EP_LD;            // floats per wave per epilogue half
  constexpr int kEpChunks = NW * EP_WAVE / 4;
  static_assert(BN != 64 || !SC || EPI == 0, "the stem modes have no BatchNorm epilogue");
  static_assert(!XF || (!SC && !Q8 && EPI != 2 && (BN >= 128 || XF == 2)), "input transform: bf16 forward");
  constexpr int kMain = NBUF * kStage > kEpChunks ? NBUF * kStage : kEpChunks;
  constexpr int kXfChunks = XF == 1 ? 2 * XFC / 4 : 0;  // fp32 scale[XFC], shift[XFC] (XF 2: registers)
  __shared__ __attribute__((aligned(16))) uint4 smem[kMain + kXfChunks];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const IgemmCls& cl = p.cls[blockIdx.z];
  // static priority for the second-dispatched half of an 8-wave workgroup (MI355X_MICROARCH.md, two
  // waves per SIMD, item 4: the younger half loses every arbitration at equal priority)
  if (NW == 8 && (p.prio & 1) && wid >= 4) __builtin_amdgcn_s_setprio(1);
  const int Mc = p.N * cl.Pc * cl.Qc;
  float* const xs = reinterpret_cast<float*>(smem + kMain);  // (XF) scale, then shift
  if constexpr (XF == 1) {
    for (int i = tid; i < p.C; i += NW * 64) {
      xs[i] = p.in_sc[i];
      xs[XFC + i] = p.in_sh[i];
    }
    __syncthreads();
  }
  // persistent mode (p.ntiles > 0, rn_set_tuning 10): each workgroup walks the tiles v = blockIdx.x +
  // k * gridDim.x (gridDim.x a multiple of 8: v stays on this XCD's contiguous tile range), so one
  // tile's output stores drain while the next tile's first K-tiles load
  const int total = p.ntiles > 0 ? p.ntiles : (int)gridDim.x;
  for (int v = blockIdx.x; v < total; v += gridDim.x) {
  const int lid = xcd_remap(v, total);
  const int mtile = lid / p.ntn;
  const int m0 = mtile * BM;
  const int n0 = (lid - mtile * p.ntn) * BN;
  if (m0 >= Mc) {  // (a dgrad parity class with fewer rows): empty BN-reduction partials
    if (EPI == 2)
      for (int e = tid; e < PR * BN; e += NW * 64) {
        const int hh = e / BN, col = n0 + e % BN;
        if (col < p.ldo && PR * mtile + hh < p.mt_max) {
          const int64_t o = ((int64_t)(blockIdx.z * p.mt_max + PR * mtile + hh) * p.ldo + col) * 2;
          p.bnred[o] = 0.f;
          p.bnred[o + 1] = 0.f;
        }
      }
    continue;
  }

  // grouped conv (ResNeXt, 64-column tile = one RN_GROUP_BLOCK): the block's columns touch groups
  // n0/gcol.., whose input channels start at cbase (dense: gcol = 2^30, cbase = 0)
  const int cbase = (n0 / p.gcol) * p.gred;
  // DMA lane -> (row 8*wid + lane/8 (+64 i), LDS slot lane&7); it fetches the source chunk that the
  // XOR read-swizzle expects in that slot
  const int lch = M32 ? (lane & 7) ^ ((4 * wid + (lane >> 4)) & 7) : (lane & 7) ^ ((lane >> 3) & 7);
  int a_row[AR], a_h[AR], a_w[AR];  // row offset of tap (0,0); its gathered coordinates
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + RPR * i + (tid >> 3);
    if (m < Mc && RPR * i + (tid >> 3) < BM) {
      const int n = fdiv(m, cl.fdPQ);
      const int rem = m - n * cl.Pc * cl.Qc;
      const int ii = fdiv(rem, cl.fdQ);
      const int jj = rem - ii * cl.Qc;
      a_h[i] = ii * p.hmul + cl.hb0 + cl.hoff0;
      a_w[i] = jj * p.wmul + cl.wb0 + cl.woff0;
      // may point before the image: masked (SC: the lane's chunk is a tap, not a channel block)
      a_row[i] = ((n * p.H + a_h[i]) * p.W + a_w[i]) * p.C + (SC ? 0 : cbase + lch * CE);
      if (SC == 2) a_row[i] = ((n * p.H + ii * p.hmul) * p.W + jj * p.wmul) * 4;  // padded image: no offsets
    } else {
      a_h[i] = -(1 << 28);  // never inside the image
      a_w[i] = 0;
      a_row[i] = 0;
    }
  }
  int b_off[BR];
  bool b_ok[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int col = n0 + RPR * i + (tid >> 3);
    b_ok[i] = col < p.K;
    b_off[i] = (b_ok[i] ? col : 0) * p.wrow + lch * CE;
  }
  const v4i rs_x = make_rsrc(p.x, (uint32_t)p.x_bytes);
  const v4i rs_w = make_rsrc(p.w, (uint32_t)p.w_bytes);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem) + wid * 1024);  // this wave's 8 rows

  const int ncb = (p.cblk + BKE - 1) / BKE;
  const int nstage = SC == 2 ? 4 : SC ? (p.rs * CE + BKE - 1) / BKE : cl.nr * cl.ns * ncb;
  int st_tr = 0, st_ts = 0, st_cb = 0, st_n = 0;
  // one K-tile's DMAs: prep() fixes the tile's uniform offsets, piece(k) issues DMA k (A rounds
  // first, then B). A tile past the range issues zero-fill DMAs (kOob) into a buffer nobody reads,
  // so the main loop has no branch around them.
  int d_toffa = 0, d_toffb = 0, d_dh = 0, d_dw = 0;
  bool d_cok = false;
  uint32_t d_la = 0;
  int d_buf = 0;
  uint32_t okb = 0;  // (XF) bit buf * AR + k: A piece k of the K-tile in buffer buf holds data
  const uint32_t dmask = (kRnDiag && (p.sched & 2)) ? 0xFFF0u : 0xFFFFFFFFu;  // diagnostic: L2-resident sources
  auto prep = [&](int buf) __attribute__((always_inline)) {
    if constexpr (SC == 2) {  // K-tile t: lane chunk lch is row 2 t + lch / 4, taps 2 (lch % 4) + {0, 1}
      const int t = st_n++;
      d_cok = t < nstage;
      d_dh = 0;  // (the padded image needs no in-image test: a_h / a_w are inside it)
      d_dw = 0;
      d_toffa = ((2 * t + (lch >> 2)) * p.W + 2 * (lch & 3)) * 4;
      d_toffb = t * BKE;
      d_la = lds0 + buf * (kStage * 16);
      return;
    }
    if constexpr (SC == 1) {  // K-tile t: lane chunk lch is tap 8 t + lch (all 8 channels of it)
      const int t = st_n++;
      const int tap = t * (BKE / CE) + lch;
      const int r = (int)fdiv((uint32_t)tap, p.fdS);
      d_cok = t < nstage && tap < p.rs;
      d_dh = r;
      d_dw = tap - r * p.S;
      d_toffa = (d_dh * p.W + d_dw) * p.C;
      d_toffb = t * BKE;
      d_la = lds0 + buf * (kStage * 16);
      return;
    }
    if constexpr (XF) {
      d_buf = buf;
      okb &= ~(((1u << AR) - 1u) << (buf * AR));
    }
    const int tr = st_tr, ts = st_ts, cb = st_cb;
    const bool live = st_n++ < nstage;
    if (++st_cb == ncb) {
      st_cb = 0;
      if (++st_ts == cl.ns) {
        st_ts = 0;
        ++st_tr;
      }
    }
    d_cok = live && cb * BKE + lch * CE < p.cblk && cbase + cb * BKE + lch * CE < p.C;
    d_dh = p.hinc * tr;
    d_dw = p.winc * ts;
    d_toffa = (d_dh * p.W + d_dw) * p.C + cb * BKE;
    d_toffb = ((cl.r0 + p.rstep * tr) * p.S + cl.s0 + p.sstep * ts) * p.cblk + cb * BKE;
    d_la = lds0 + buf * (kStage * 16);
  };
  // the A rows past a 224-row tile's last (the 256-row A region's last 32 rows) are never read: a wave
  // whose 8 rows of a DMA round lie there skips that piece (8-wave tiles: 4 of the K-tile's 64 pieces;
  // at most one per wave and K-tile)
  static_assert(BMA - BM <= RPR, "at most one skipped A piece per wave");
  const bool skip_last = 8 * wid + RPR * (AR - 1) >= BM && !(p.prio & 2);  // (rn_set_tuning 20 bit 2: no skip)
  auto piece = [&](int k) __attribute__((always_inline)) {
    if (k == AR - 1 && skip_last) return;
    if (k < AR) {
      const bool ok = W4 ? d_cok && a_h[k] >= 0
                         : d_cok && (unsigned)(a_h[k] + d_dh) < (unsigned)p.H && (unsigned)(a_w[k] + d_dw) < (unsigned)p.W;
      if constexpr (XF) okb |= (uint32_t)ok << (d_buf * AR + k);
      dma16_asm(rs_x, d_la + k * (RPR * 128), ok ? ((uint32_t)((a_row[k] + d_toffa) * ES) & dmask) : kOob);
    } else {
      const int i = k - AR;
      dma16_asm(rs_w, d_la + BMA * 128 + i * (RPR * 128),
                (d_cok && b_ok[i]) ? ((uint32_t)((b_off[i] + d_toffb) * ES) & dmask) : kOob);
    }
  };
  // diagnostic (rn_set_tuning 7 bit 8): no DMAs inside the main loop (wrong results; isolates their cost)
  const bool loop_dma = !(kRnDiag && (p.sched & 8));
  auto lpiece = [&](int k) __attribute__((always_inline)) {
    if (loop_dma) piece(k);
  };
  auto issue = [&](int buf) __attribute__((always_inline)) {
    prep(buf);
#pragma unroll
    for (int k = 0; k < LPT; ++k) piece(k);
  };

  AccT acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = AccT{};

  // the MFMAs of K-tile `buf`, with the next K-tile's DMAs between the first MFMA groups
  // (inline asm is a scheduling boundary: each DMA's address arithmetic overlaps the MFMAs around it)
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const uint4* As = smem + buf * kStage;
    const uint4* Bs = As + BMA * 8;
    // k-steps per K-tile: 4 of 16 (32x32x16: lane half h = lane >> 5 holds chunk 2 ks + h of its
    // row) or 2 of 32 (16x16x32: lane quarter q = lane >> 4 holds chunk 4 ks + q). Fragments are
    // double-buffered in registers: k-step ks + 1 is read while ks multiplies.
    constexpr int KS = M32 ? 4 : 2;
    uint4 af[2][MI], bfr[2][NI];
    // (GD) does k-step ks meet column sub-block j?
    auto live = [](int ks, int j) __attribute__((always_inline)) {
      return !GD || (M32 ? (ks >> 1) == j : (j >> 1) == ks);
    };
    auto ldf = [&](int ks) __attribute__((always_inline)) {
      const int kc = M32 ? 2 * ks + (lane >> 5) : 4 * ks + (lane >> 4);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (!live(ks, j)) continue;
        const int row = wn * WN + j * FM + (lane & (FM - 1));
        bfr[ks & 1][j] = Bs[row * 8 + (M32 ? swz32(row, kc) : swz(row, kc))];
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * WM + i * FM + (lane & (FM - 1));
        af[ks & 1][i] = As[row * 8 + (M32 ? swz32(row, kc) : swz(row, kc))];
      }
    };
    ldf(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) ldf(ks + 1);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if (!live(ks, j)) continue;
          if constexpr (Q8) {
            const uint4 a8 = af[ks & 1][i], b8 = bfr[ks & 1][j];
            acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(*reinterpret_cast<const v4i*>(&a8),
                                                               *reinterpret_cast<const v4i*>(&b8), acc[i][j], 0, 0, 0);
          } else if constexpr (M32) {
            mfma32(acc[i][j], af[ks & 1][i], bfr[ks & 1][j]);
          } else {
            mfma_slab<bf16_t>(acc[i][j], af[ks & 1][i], bfr[ks & 1][j]);
          }
        }
        // 2 buffers: the DMAs over the first half of the K-tile's MFMA groups, so they have the
        // longest to land; 3 buffers (one more K-tile in flight): spread over all of them
        constexpr int G = NBUF == 1 ? 0 : NBUF == 2 ? KS / 2 * MI : KS * MI;
        const int g = ks * MI + i;
        if (g < G) {
#pragma unroll
          for (int q = g * LPT / G; q < (g + 1) * LPT / G; ++q) lpiece(q);
        }
      }
    }
  };

  // (XF 2: C = 64, one channel block: this thread's chunk is always channels lch * 8.., its scale / shift
  // two registers each, no LDS table -- the 64-column tile keeps two workgroups per CU)
  float xa[XF == 2 ? 8 : 1], xb[XF == 2 ? 8 : 1];
  if constexpr (XF == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xa[e] = p.in_sc[lch * CE + e];
      xb[e] = p.in_sh[lch * CE + e];
    }
  }
  // (XF) this thread's landed A chunks of the K-tile in buffer buf, channel block cb, rewritten in place
  auto xform = [&](int buf, int cb) __attribute__((always_inline)) {
    float a[8], b[8];
    if constexpr (XF == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[e] = xa[e];
        b[e] = xb[e];
      }
    } else {
      const int c0 = min(cb * BKE + lch * CE, p.C - CE);  // (clamped: a chunk past C was zero-filled)
      *reinterpret_cast<float4*>(a) = *reinterpret_cast<const float4*>(xs + c0);
      *reinterpret_cast<float4*>(a + 4) = *reinterpret_cast<const float4*>(xs + c0 + 4);
      *reinterpret_cast<float4*>(b) = *reinterpret_cast<const float4*>(xs + XFC + c0);
      *reinterpret_cast<float4*>(b + 4) = *reinterpret_cast<const float4*>(xs + XFC + c0 + 4);
    }
#pragma unroll
    for (int k = 0; k < AR; ++k) {
      uint4* cp = smem + buf * kStage + k * (RPR * 8) + tid;
      float f[8];
      chunk_to_f(*cp, f, (const bf16_t*)nullptr);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], a[e], b[e]), 0.f);
      const uint4 o = f_to_chunk(f, (const bf16_t*)nullptr);
      *cp = ((okb >> (buf * AR + k)) & 1u) ? o : make_uint4(0, 0, 0, 0);
    }
  };
  int xf_cb = 0;

#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(s);
  for (int t = 0; t < nstage; ++t) {
    if constexpr (NBUF == 1) {  // one buffer: refilled once every wave is done reading it
      if (t > 0) __syncthreads();
      issue(0);
      wait_vmcnt<0>();
      if constexpr (XF) {
        xform(0, xf_cb);
        if (++xf_cb == ncb) xf_cb = 0;
      }
      __syncthreads();
      compute(0);
      continue;
    }
    // K-tile t has landed for this thread once at most the later K-tiles' DMAs are outstanding
    if (!(kRnDiag && (p.sched & 4))) {  // (diagnostic bit 4: no wait, no barrier -- wrong results)
      if (NBUF == 3) {
        if (skip_last) wait_vmcnt<(LPT > 0 ? LPT - 1 : 0)>();  // (one piece fewer per K-tile)
        else wait_vmcnt<LPT>();
      } else {
        wait_vmcnt<0>();
      }
      if constexpr (XF) {
        xform(t % NBUF, xf_cb);
        if (++xf_cb == ncb) xf_cb = 0;
      }
      __syncthreads();  // ... for every thread; and every wave is done reading the buffer refilled next
    }
    prep((t + NBUF - 1) % NBUF);
    if (kRnDiag && (p.sched & 1)) __builtin_amdgcn_s_setprio(1);
    compute(t % NBUF);
    if (kRnDiag && (p.sched & 1)) __builtin_amdgcn_s_setprio(0);
  }
  wait_vmcnt<0>();  // the zero-fill DMAs past the range land before the epilogue reuses the buffers
  __syncthreads();  // the epilogue reuses the staging buffers
  if (kRnDiag && (p.sched & 16)) {  // diagnostic (rn_set_tuning 7 bit 16): no epilogue, one store per wave keeps
                       // the accumulators live (wrong results; isolates the epilogue's cost)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) t += (float)acc[i][j][0];
    if (lane == 0) reinterpret_cast<float*>(p.y)[v] = t;  // one slot per tile (persistent mode walks several)
    continue;
  }

  // ---- epilogue: per wave, 64 accumulator rows at a time through LDS, then 16-byte row chunks
  constexpr int CPR = WN / 8;  // 8-column output chunks per wave row
  constexpr int AW = sizeof(OutT) / 2;  // 16-byte pieces per 8-column chunk (bf16 1, fp32 2)
  const float qscale = Q8 ? p.qunit_x[0] * p.qunit_w[0] : 1.f;
  float* ep = reinterpret_cast<float*>(smem) + wid * EP_WAVE;
  const OutT* __restrict__ ag = reinterpret_cast<const OutT*>(p.add);
  OutT* __restrict__ yg = reinterpret_cast<OutT*>(p.y);
  const int cc = lane % CPR;
  const int col0 = n0 + wn * WN + cc * 8;
  const bool half_ok = m0 + wm * WM < Mc;  // this wave row holds at least one output row
  // BatchNorm partials of this lane's 8 columns (EPI 1: S1, S2 about the pivot; EPI 2: sum dz,
  // sum dz * (x - mean)), over its rows; the lanes sharing a column chunk are summed at the end.
  // EPI 3 keeps its coefficients in the same registers: s1 = A, s2 = mean(dz), piv = A2, r_mu = mean.
  constexpr int NS = EPI ? 8 : 1;
  constexpr int NM = MM ? 8 : 1;  // (MM: running max of sgn * the stored values)
  float s1[NS], s2[NS], piv[NS], r_mu[NS], r_sc[NS], r_sh[NS], mxv[NM], sgn[NM];
  constexpr bool want_mm = MM;
#pragma unroll
  for (int e = 0; e < NM; ++e) mxv[e] = -INFINITY;
  if constexpr (MM) {  // the sign vector's 8 values in two 16-byte loads (host: 16-byte aligned, K % 8 == 0)
    float4 g0 = make_float4(1.f, 1.f, 1.f, 1.f), g1 = g0;
    if (p.mm_sign && col0 < p.K) {
      g0 = reinterpret_cast<const float4*>(p.mm_sign + col0)[0];
      g1 = reinterpret_cast<const float4*>(p.mm_sign + col0)[1];
    }
    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int e = 0; e < NM; ++e) sgn[e] = gv[e] < 0.f ? -1.f : 1.f;
  } else {
#pragma unroll
    for (int e = 0; e < NM; ++e) sgn[e] = 1.f;
  }
#pragma unroll
  for (int e = 0; e < NS; ++e) {
    s1[e] = s2[e] = piv[e] = r_mu[e] = r_sc[e] = r_sh[e] = 0.f;
    if constexpr (EPI == 2 || EPI == 3) {
      const bool okc = col0 + e < p.K;
      r_sc[e] = okc ? p.bn_sc[col0 + e] : 0.f;
      r_sh[e] = okc ? p.bn_sh[col0 + e] : 0.f;
      if constexpr (EPI == 2) {
        r_mu[e] = okc ? p.bn_mean[col0 + e] : 0.f;
      } else if (okc) {
        const float4 cf = reinterpret_cast<const float4*>(p.bn_coef)[col0 + e];
        s1[e] = cf.x;
        s2[e] = cf.y;
        piv[e] = cf.z;
        r_mu[e] = cf.w;
      }
    }
  }
  const bf16_t* __restrict__ bxg = reinterpret_cast<const bf16_t*>(p.bn_x);
  const float clipt = CLIP ? *p.bn_clip : 0.f;  // (EPI 4: a folded quantizer clip)
  // (EPI 4, a quantizer pair: the two quantizers of one BN+ReLU output, symbol/resnet_int8.py's stage-first
  // units. This dgrad's own gradient takes clip 1, the add operand -- the other quantizer's stored gradient
  // -- clip 2; the stored value is their clipped sum, rounded once, as rn_bn.hip's relu_clip2_dz forms
  // it, and the reduction reads it with the ReLU mask only)
  const bool qpair = CLIP && p.bn_clip2 != nullptr;
  const float clipt2 = qpair ? *p.bn_clip2 : 0.f;
#pragma unroll
  for (int h = 0; h < NCH; ++h) {
    constexpr int kLast = WM - 64 * (NCH - 1);  // rows of the last chunk (48 for 112-row waves)
    const int rows_h = h + 1 < NCH ? 64 : kLast;
    int64_t off[CPR];  // this lane's rows: lane / CPR + (64 / CPR) k
    uint4 addv[CPR][AW];
    constexpr bool XP = EPI == 2 || EPI == 3;
    uint4 xpre[XP ? CPR : 1];  // BN input at the same positions (EPI 2 / 3), loaded with the residual
#pragma unroll
    for (int k = 0; k < CPR; ++k) {
      const int r = lane / CPR + (64 / CPR) * k;
      const int m = m0 + wm * WM + h * 64 + r;
      off[k] = -1;
#pragma unroll
      for (int u = 0; u < AW; ++u) addv[k][u] = make_uint4(0, 0, 0, 0);
      if constexpr (XP) xpre[k] = make_uint4(0, 0, 0, 0);
      if (m < Mc && col0 < p.K && r < rows_h) {
        const int n = fdiv(m, cl.fdPQ);
        const int rem = m - n * cl.Pc * cl.Qc;
        const int ii = fdiv(rem, cl.fdQ);
        const int jj = rem - ii * cl.Qc;
        off[k] = ((int64_t)(n * p.P + cl.a + p.ostep_h * ii) * p.Q + cl.b + p.ostep_w * jj) * p.ldo + col0;
        const bool eld = !(kRnDiag && (p.sched & 256));  // (diagnostic bit 256: no epilogue loads)
        if (ag && col0 + 8 <= p.K && eld)
#pragma unroll
          for (int u = 0; u < AW; ++u) addv[k][u] = reinterpret_cast<const uint4*>(ag + off[k])[u];
        if constexpr (XP)
          if (col0 + 8 <= p.K && eld) xpre[k] = *reinterpret_cast<const uint4*>(bxg + off[k]);
      }
    }
    // Each wave stages through its own LDS region, so the epilogue needs no block barrier -- a wave's
    // LDS accesses execute in order, and its reads of a half have returned before the next half's
    // writes issue -- except where wave row 1 reads wave row 0's pivot row (EPI 1 on paired rows).
    // rn_set_tuning 16 = 1: block barriers everywhere (the previous form, for A/B).
    constexpr bool XW = EPI == 1 && PAIR;
    const bool blk_sync = XW || p.epi_sync;
    if (h > 0 && blk_sync) __syncthreads();  // the first half's staged rows have been read
    if constexpr (M32) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            ep[(i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * EP_LD + j * 32 + (lane & 31)] =
                acc[h * 2 + i][j][e];
    } else if (kRnDiag && (p.sched & 64)) {  // diagnostic (rn_set_tuning 7 bit 64): no staging writes (the
                                           // accumulators kept live, the staged values stale: wrong results)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (h * 4 + i < MI)
#pragma unroll
          for (int j = 0; j < NI; ++j) asm volatile("" ::"v"(acc[h * 4 + i][j]));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (h * 4 + i < MI)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              ep[(i * 16 + (lane >> 4) * 4 + e) * EP_LD + j * 16 + (lane & 15)] =
                  Q8 ? (float)acc[h * 4 + i][j][e] * qscale : (float)acc[h * 4 + i][j][e];
    }
    if (blk_sync) __syncthreads();
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's staged rows have landed
    if constexpr (EPI == 1) {
      if (h == 0) {  // pivot: the first (rounded) conv value of each column in the tile's first wave
                     // row (PAIR: both wave rows use it, so their sums add), else in this wave row
        const float* ep0 = PAIR ? reinterpret_cast<const float*>(smem) + wn * EP_WAVE : ep;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          piv[e] = to_f(from_f<OutT>(ep0[cc * 8 + e]));
      }
    }
#pragma unroll
    for (int k = 0; k < CPR; ++k) {
      if (off[k] < 0) continue;
      const int r = lane / CPR + (64 / CPR) * k;
      float v[8];
      if (kRnDiag && (p.sched & 512)) {  // (diagnostic bit 512: no staging reads -- stale values)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (float)(r + e);
      } else {
        *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(ep + r * EP_LD + cc * 8);
        *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(ep + r * EP_LD + cc * 8 + 4);
      }
      if (col0 + 8 <= p.K) {
        if constexpr (EPI == 3) {
          // the BatchNorm(+ReLU) backward applied to the gradient as rn_conv_bwd_data would store it,
          // exactly as bn_bwd_apply_kernel (rn_bn.hip) computes it from the stored gradient
          float g[8], xv[8], a[8];
          chunk_to_f(f_to_chunk(v, (const bf16_t*)nullptr), g, (const bf16_t*)nullptr);
          chunk_to_f(xpre[XP ? k : 0], xv, (const bf16_t*)nullptr);
          if (ag) chunk_to_f(addv[k][0], a, (const bf16_t*)nullptr);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = p.bn_relu ? g[e] * (fmaf(xv[e], r_sc[e], r_sh[e]) > 0.f ? 1.f : 0.f) : g[e];
            float w = s1[e] * (dz - s2[e]) - piv[e] * (xv[e] - r_mu[e]);
            if (ag) w += a[e];
            v[e] = w;
          }
        } else if (CLIP && qpair) {  // c1 * bf16(own) + c2 * add, c = [bf16(BN output) < t]
          float a[8], xv[8];
          chunk_to_f(addv[k][0], a, (const bf16_t*)nullptr);
          chunk_to_f(xpre[XP ? k : 0], xv, (const bf16_t*)nullptr);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float y = to_f(from_f<bf16_t>(fmaf(xv[e], r_sc[e], r_sh[e])));
            const float own = to_f(from_f<bf16_t>(v[e]));
            v[e] = (y < clipt ? own : 0.f) + (y < clipt2 ? a[e] : 0.f);
          }
        } else if (ag) {
          float a[8];
#pragma unroll
          for (int u = 0; u < AW; ++u) chunk_to_f(addv[k][u], a + u * (8 / AW), (const OutT*)nullptr);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += a[e];
        }
        uint4 out[AW];
#pragma unroll
        for (int u = 0; u < AW; ++u) out[u] = f_to_chunk(v + u * (8 / AW), (const OutT*)nullptr);
        if (yg && (!(kRnDiag && (p.sched & 32)) || (out[0].x & 0xFFFF) == 0x7FC1))  // (EPI 2 may only reduce;
                                                                                  // diagnostic bit 32: no stores)
        {
          if (p.nt_store) {  // streaming hint: fewer dirty lines left for the end-of-kernel L2 write-back
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int u = 0; u < AW; ++u) {
              const u32x4 w = {out[u].x, out[u].y, out[u].z, out[u].w};
              __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(yg + off[k]) + u);
            }
          } else {
#pragma unroll
            for (int u = 0; u < AW; ++u) reinterpret_cast<uint4*>(yg + off[k])[u] = out[u];
          }
        }
        if (EPI != 1 && EPI != 2) {
        } else if (kRnDiag && (p.sched & 128)) {  // diagnostic (bit 128): no BatchNorm partial math (wrong results)
        } else if constexpr (EPI == 1 || EPI == 2) {  // on the stored (rounded) values, as a separate pass would read them
          float g[8];
#pragma unroll
          for (int u = 0; u < AW; ++u) chunk_to_f(out[u], g + u * (8 / AW), (const OutT*)nullptr);
          if constexpr (EPI == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = g[e] - piv[e];
              s1[e] += d;
              s2[e] = fmaf(d, d, s2[e]);
            }
            if (want_mm)
#pragma unroll
              for (int e = 0; e < NM; ++e) mxv[e] = fmaxf(mxv[e], sgn[e] * g[e]);
          } else {
            float xv[8];
            chunk_to_f(xpre[XP ? k : 0], xv, (const bf16_t*)nullptr);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float dz = (!p.bn_relu || fmaf(xv[e], r_sc[e], r_sh[e]) > 0.f) ? g[e] : 0.f;
              if constexpr (CLIP)  // the quantizer's straight-through clip on the stored BN output
                if (!qpair && !(to_f(from_f<bf16_t>(fmaf(xv[e], r_sc[e], r_sh[e]))) < clipt)) dz = 0.f;
              s1[e] += dz;
              s2[e] = fmaf(dz, xv[e] - r_mu[e], s2[e]);
            }
          }
        }
      } else if (yg) {  // (ragged columns: never with EPI 3, whose channels come in whole chunks)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col0 + e < p.K) {
            float o = v[e];
            if (ag) o += to_f(ag[off[k] + e]);
            yg[off[k] + e] = from_f<OutT>(o);
          }
      }
    }
  }
  if constexpr (EPI == 1 || EPI == 2) {
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (want_mm)
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < NM; ++e) mxv[e] = fmaxf(mxv[e], __shfl_xor(mxv[e], o, 64));
    if constexpr (PAIR) {  // wave row 1 hands its sums (and max / min) to wave row 0 (same columns)
      float* xch = reinterpret_cast<float*>(smem) + wn * (CPR * 32);
      __syncthreads();  // every wave is done reading the epilogue staging
      if (wm == 1 && lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xch[lane * 32 + e] = s1[e];
          xch[lane * 32 + 8 + e] = s2[e];
        }
        if (want_mm)
#pragma unroll
          for (int e = 0; e < NM; ++e) xch[lane * 32 + 16 + e] = mxv[e];
      }
      __syncthreads();
      if (wm == 0 && lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] += xch[lane * 32 + e];
          s2[e] += xch[lane * 32 + 8 + e];
        }
        if (want_mm)
#pragma unroll
          for (int e = 0; e < NM; ++e) mxv[e] = fmaxf(mxv[e], xch[lane * 32 + 16 + e]);
      }
    }
    if (lane < CPR && (!PAIR || wm == 0)) {
      const int c0 = n0 + wn * WN + lane * 8;
      const int blk = PR * mtile + (PAIR ? 0 : wm);  // one partial per tile (PAIR) or wave row
      const bool rows_ok = PAIR || half_ok;         // (PAIR: wave row 0 always holds rows)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = c0 + e;
        if (col >= p.ldo) continue;
        const bool okc = col < p.K;
        if constexpr (EPI == 1) {
          if (rows_ok) {
            float* dst = p.stats + (int64_t)blk * 3 * p.ldo + col;
            dst[0] = okc ? s1[e] : 0.f;
            dst[p.ldo] = okc ? s2[e] : 0.f;
            dst[2 * p.ldo] = piv[e];
            if (want_mm)
              p.stats_mm[(int64_t)blk * p.ldo + col] = okc ? sgn[e < NM ? e : 0] * mxv[e < NM ? e : 0] : 0.f;
          }
        } else if (blk < p.mt_max) {  // (a half past the class's rows may lie past its partial slots)
          const int64_t o = ((int64_t)(blockIdx.z * p.mt_max + blk) * p.ldo + col) * 2;
          p.bnred[o] = (rows_ok && okc) ? s1[e] : 0.f;
          p.bnred[o + 1] = (rows_ok && okc) ? s2[e] : 0.f;
        }
      }
    }
  }
  __syncthreads();  // (persistent) the epilogue's LDS reads end before the next tile's DMAs
  }
}

// ------------------------------------------------------------------------------ wgrad
struct WgradArgs {
  const void* x;   // NHWC gathered (B operand)
  const void* dy;  // [M][ldy] (A operand)
  float* dw;       // [K][ldw]
  int N, H, W, C, P, Q, K, ldy, R, S, sh, sw, ph, pw;
  int ncol_load;   // R*S*C
  int ncol;        // valid columns of dw (R*S*c_real)
  int ldw;
  int M;
  int m_per_split;
  int grouped, gk, gc, cblk;  // grouped: rows / channels per group, channels per row block
  int creal;                  // logical input channels (< C: padded stride, dw keeps c < creal)
  int nct, nkt;               // column tiles, k tiles (grid = splits * nkt * nct)
  int diag_noepi;             // diagnostic (rn_set_tuning 6, bits): 1 skip the dW epilogue, 2 / 4 (wgrad_big_kernel) no loop DMAs / waits
  int x_bytes, dy_bytes;      // (wgrad_big_kernel) the operands' buffer descriptor sizes
  int p4;                     // the stem's padded NHWC4 image (rn_stem_prepare_p4): column = (r*8 + s)*4 + c,
                              // r, s < 8; dW keeps r < R, s < S, c < creal ([K][R][S][creal])
  int gspread;                // (gdiag) the diagonal blocks spread over all four waves
  int gdiag;                  // grouped zero-block skip (bf16, rn_set_tuning 14): 16-row blocks per group
                              // span (1: <= 16 channels per group, 2: 32); 0 = off
  float* slab;                // nullable (LDS-DMA kernels): the split's tile stored into slab[split][K][ldw]
                              // (no atomics; wgrad_slab_reduce_kernel sums the splits into dw)
  const float* in_sc;         // nullable: BN+ReLU applied to the gathered x while staging
  const float* in_sh;
  const float* xunit;         // (wgrad_big_kernel I8X) x holds int8 codes: dW = unit * sum dy * code
  FastDiv fdQ, fdPQ, fdC, fdS;  // fdC divides by cblk (dense: C)
};

// 16-byte chunk swizzle of an LDS image whose rows are read 4-at-a-time by
// ds_read_b64_tr_b16 (rows 8g+4h+q): keeps the 8 rows of a 32-lane half on distinct slots.
__device__ __forceinline__ int swz_tr(int row) { return 2 * ((row & 3) | (((row >> 3) & 1) << 2)); }
// (int8 B images, read 8 rows per ds_read_b64_tr_b8: rows 8 g .. 8 g + 7 on 8 distinct chunks)
__device__ __forceinline__ int swz_tr8(int row) { return row & 7; }
// 8 int8 codes (two dwords, bytes in row order) -> 8 bf16 of the same integers (exact): bias to unsigned,
// the byte conversions, minus the bias, then the fp32 high halves
__device__ __forceinline__ v8s i8x8_to_bf16(v2i v) {
  uint32_t o[4];
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const uint32_t u = (uint32_t)v[w] ^ 0x80808080u;
    const float f0 = (float)(u & 0xFFu) - 128.f, f1 = (float)((u >> 8) & 0xFFu) - 128.f;
    const float f2 = (float)((u >> 16) & 0xFFu) - 128.f, f3 = (float)(u >> 24) - 128.f;
    o[2 * w] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
    o[2 * w + 1] = __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u);
  }
  v8s r;
  __builtin_memcpy(&r, o, 16);
  return r;
}

template <typename T, int BMK, int BNC, bool XF = false, bool GW = false>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs p) {
  constexpr int CE = 16 / sizeof(T);
  constexpr int BKM = 128 / sizeof(T);        // m rows per stage
  constexpr int A_CPR = BMK * sizeof(T) / 16; // chunks per A row
  constexpr int B_CPR = BNC * sizeof(T) / 16;
  constexpr int A_CH = BKM * A_CPR / 256;
  constexpr int B_CH = BKM * B_CPR / 256;
  constexpr int A_RSTEP = 256 / A_CPR;
  constexpr int B_RSTEP = 256 / B_CPR;
  constexpr int MI = BMK / 32;
  constexpr int NI = BNC / 32;
  constexpr int A_SZ = BKM * A_CPR;  // chunks
  constexpr int B_SZ = BKM * B_CPR;
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * (A_SZ + B_SZ)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // 1-D grid over (m split, k tile, column tile), column fastest, XCD-remapped: the tiles of one
  // m range (which re-read the same dy rows and x pixels) share an L2
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_split = p.nct * p.nkt;
  const int zs = lid / per_split;
  const int rem = lid - zs * per_split;
  const int kt = rem / p.nct;
  const int n0 = (rem - kt * p.nct) * BNC;  // dw column tile
  const int k0 = kt * BMK;                  // dw row tile (output channels)
  const int mbeg = zs * p.m_per_split;
  const int mend = min(p.M, mbeg + p.m_per_split);
  if (mbeg >= mend) return;
  const int cbase = p.grouped ? (k0 / p.gk) * p.gc : 0;

  const T* __restrict__ xg = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ dyg = reinterpret_cast<const T*>(p.dy);

  // A assignment: chunk column a_c, rows (tid / A_CPR) + A_RSTEP*i
  const int a_c = tid % A_CPR;
  const int a_k = k0 + a_c * CE;
  const bool a_kok = a_k < p.ldy;
  // B assignment: fixed column chunk -> (tap r,s ; channel c)
  const int b_c = tid % B_CPR;
  const int bcol = n0 + b_c * CE;
  bool b_cok = bcol < p.ncol_load;
  int b_r = 0, b_s = 0, b_ch = 0;
  if (b_cok) {
    const int tap = fdiv(bcol, p.fdC);
    b_ch = cbase + bcol - tap * p.cblk;
    b_r = fdiv(tap, p.fdS);
    b_s = tap - b_r * p.S;
    b_cok = b_ch < p.C;  // a grouped block may run past the last group
  }
  const int b_hoff = b_r - p.ph, b_woff = b_s - p.pw;
  // BN+ReLU input transform: this thread's column chunk (channels b_ch..) is fixed for the kernel
  float tsc[XF ? CE : 1], tsh[XF ? CE : 1];
  if constexpr (XF) {
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      tsc[e] = b_cok ? p.in_sc[b_ch + e] : 0.f;
      tsh[e] = b_cok ? p.in_sh[b_ch + e] : 0.f;
    }
  }

  uint4 ra[A_CH], rb[B_CH];
  uint32_t xok = 0;  // (XF) B chunk i holds an input pixel: transformed when stored to LDS
  auto load_stage = [&](int mb) {
    xok = 0;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = mb + tid / A_CPR + A_RSTEP * i;
      if (a_kok && m < mend)
        ra[i] = *reinterpret_cast<const uint4*>(dyg + (int64_t)m * p.ldy + a_k);
      else
        ra[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int m = mb + tid / B_CPR + B_RSTEP * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b_cok && m < mend) {
        const int n = fdiv(m, p.fdPQ);
        const int rem = m - n * p.P * p.Q;
        const int pp = fdiv(rem, p.fdQ);
        const int qq = rem - pp * p.Q;
        const int hin = pp * p.sh + b_hoff;
        const int win = qq * p.sw + b_woff;
        if ((unsigned)hin < (unsigned)p.H && (unsigned)win < (unsigned)p.W) {
          v = *reinterpret_cast<const uint4*>(
              xg + ((int64_t)(n * p.H + hin) * p.W + win) * p.C + b_ch);
          xok |= 1u << i;
        }
      }
      rb[i] = v;
    }
  };
  auto store_stage = [&](int buf) {
    uint4* As = smem + buf * (A_SZ + B_SZ);
    uint4* Bs = As + A_SZ;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = tid / A_CPR + A_RSTEP * i;
      As[row * A_CPR + (a_c ^ (swz_tr(row) & (A_CPR - 1)))] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = tid / B_CPR + B_RSTEP * i;
      uint4 v = rb[i];
      if constexpr (XF) {  // after the MFMA phase: the loads were in flight under it
        float f[CE];
        chunk_to_f(v, f, (const T*)nullptr);
#pragma unroll
        for (int e = 0; e < CE; ++e) f[e] = fmaxf(fmaf(f[e], tsc[e], tsh[e]), 0.f);
        v = ((xok >> i) & 1u) ? f_to_chunk(f, (const T*)nullptr) : make_uint4(0, 0, 0, 0);
      }
      Bs[row * B_CPR + (b_c ^ (swz_tr(row) & (B_CPR - 1)))] = v;
    }
  };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  // grouped, equal rows and channels per group (<= 32, the 64 x 64 tile = one RN_GROUP_BLOCK): the
  // 16 x 16 block (16-row block rb of k, 16-column block cb of c) is nonzero only when both lie in
  // the same group span: only the two diagonal 32 x 32 blocks are computed, wave (wm, wn) taking
  // diagonal block wm over the stage's 32-row slab wn (the two partials of a block meet in the
  // epilogue's atomic adds), and inside it the off-diagonal 16 x 16 blocks are skipped
  const int gd = GW && sizeof(T) == 2 ? p.gdiag : 0;  // (GW: the grouped instantiation only)
  const bool spread = gd && p.gspread;                 // rn_set_tuning 14 = 2: two waves idle instead
  const int wnE = spread ? wm : wn;                    // the wave's column half
  const bool wave_live = !gd || spread || wm == wn;
  auto live = [&](int i, int j) __attribute__((always_inline)) {
    return !gd || (wm * MI + i) / gd == (wnE * NI + j) / gd;
  };

  const int nstage = (mend - mbeg + BKM - 1) / BKM;
  load_stage(mbeg);
  store_stage(0);
  __syncthreads();
  for (int t = 0; t < nstage; ++t) {
    const bool more = t + 1 < nstage;
    if (more) load_stage(mbeg + (t + 1) * BKM);
    const uint4* As = smem + (t & 1) * (A_SZ + B_SZ);
    const uint4* Bs = As + A_SZ;
    if constexpr (sizeof(T) == 2) {
      if (wave_live) {
      // 2 slabs of 32 m per stage; per slab each lane needs rows 8g+j (j=0..7) at its column.
      const char* Ab = reinterpret_cast<const char*>(As);
      const char* Bb = reinterpret_cast<const char*>(Bs);
      const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
#pragma unroll
      for (int slab = 0; slab < 2; ++slab) {
        if (spread && slab != wn) continue;  // (grouped: one slab per wave)
        v8s af[MI], bfv[NI];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = slab * 32 + 8 * g + 4 * h + q;
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int col = wm * (BMK / 2) + i * 16 + 4 * pp;  // element column
            const int cch = (col * 2) >> 4;
            const int byte = row * (A_CPR * 16) + ((cch ^ (swz_tr(row) & (A_CPR - 1))) << 4) + ((col * 2) & 15);
            v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s*)(Ab + byte));
            af[i][4 * h + 0] = v[0];
            af[i][4 * h + 1] = v[1];
            af[i][4 * h + 2] = v[2];
            af[i][4 * h + 3] = v[3];
          }
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int col = wnE * (BNC / 2) + j * 16 + 4 * pp;
            const int cch = (col * 2) >> 4;
            const int byte = row * (B_CPR * 16) + ((cch ^ (swz_tr(row) & (B_CPR - 1))) << 4) + ((col * 2) & 15);
            v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s*)(Bb + byte));
            bfv[j][4 * h + 0] = v[0];
            bfv[j][4 * h + 1] = v[1];
            bfv[j][4 * h + 2] = v[2];
            bfv[j][4 * h + 3] = v[3];
          }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            if (live(i, j)) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
      }
    } else {
      // f32: 16x16x4 steps; lane holds A[k=col l&15][m = 4s + (l>>4)].
      const float* Af = reinterpret_cast<const float*>(As);
      const float* Bf = reinterpret_cast<const float*>(Bs);
#pragma unroll 4
      for (int s4 = 0; s4 < BKM / 4; ++s4) {
        const int row = 4 * s4 + (lane >> 4);
        float a[MI], b[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int col = wm * (BMK / 2) + i * 16 + (lane & 15);
          const int cch = col >> 2;
          a[i] = Af[(row * A_CPR + (cch ^ (swz_tr(row) & (A_CPR - 1)))) * 4 + (col & 3)];
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int col = wn * (BNC / 2) + j * 16 + (lane & 15);
          const int cch = col >> 2;
          b[j] = Bf[(row * B_CPR + (cch ^ (swz_tr(row) & (B_CPR - 1)))) * 4 + (col & 3)];
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store_stage((t + 1) & 1);
    __syncthreads();
  }

  // epilogue: D[row = k][col] -> atomic add into dw
  if (kRnDiag && (p.diag_noepi & 1)) {  // keep the accumulators live without touching memory
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 12345.678f) p.dw[0] = s;
    return;
  }
  // (deterministic mode, p.slab: this split's partial into slab[zs][K][ldw] -- every element of a
  // split is produced by exactly one wave of one block -- and wgrad_slab_reduce_kernel sums the splits
  // in order)
  float* const dst = p.slab ? p.slab + (int64_t)zs * p.K * p.ldw : p.dw;
  auto put = [&](int64_t i, float v) __attribute__((always_inline)) {
    if (p.slab) dst[i] = v;
    else atomicAdd(dst + i, v);
  };
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + wm * (BMK / 2) + i * 16 + (lane >> 4) * 4 + e;
      if (k >= p.K) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wnE * (BNC / 2) + j * 16 + (lane & 15);
        if (!p.grouped && p.creal == p.C) {
          if (col < p.ncol) put((int64_t)k * p.ldw + col, acc[i][j][e]);
        } else if (!p.grouped) {  // padded channels (the stem's 3 of 8): keep c < c_real
          if (col < p.ncol_load) {
            const int tap = fdiv(col, p.fdC);
            const int c = col - tap * p.C;
            if (c < p.creal) put((int64_t)k * p.ldw + tap * p.creal + c, acc[i][j][e]);
          }
        } else if (col < p.ncol_load) {  // keep the block-diagonal part: channel in k's group
          const int tap = fdiv(col, p.fdC);
          const int c = cbase + col - tap * p.cblk;
          const int g = k / p.gk;
          if (c / p.gc == g) put((int64_t)k * p.ldw + tap * p.gc + (c - g * p.gc), acc[i][j][e]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------ wgrad, big tiles
// dW[k0..+BMK][n0..+256] += dy^T * gather(x) over one M range, 8 waves (2 along k x 4 along the
// columns), bf16, dense, unpadded channels. Both operands are staged by inline-asm LDS-DMA into
// [64 m][row] images whose 16-byte chunks are XOR-swizzled (swz_tr) by choosing each lane's SOURCE
// chunk, and read with ds_read_b64_tr_b16 as in wgrad_kernel. NBUF buffers, NBUF-1 M-tiles in flight.
// BNC = 256: 8 waves, one workgroup per CU; BNC = 128: 4 waves (2 x 2, each 64-128 rows x 64
// columns), two workgroups per CU.
// XF (1x1 convolutions only: no halo, so every B element is a real input pixel or a row past the
// M range, whose dy row is zero): the producing BatchNorm+ReLU applied to the B fragments after
// their transposed read. A lane's B fragment j holds one output column (= input channel) for the
// whole kernel, so its scale / shift are two registers; max(x*sc + sh, 0) rounded to bf16 as
// bn_apply_kernel does.
// I8X: x holds the int8 codes of an activation Quantization_int8 (symbol/resnet_int8.py; the input of an
// int8 convolution, whose fake-quantized values x = unit * code the weight gradient multiplies): the B
// image holds the bytes (16 channels per 16-byte chunk, half the LDS and HBM bytes), read with
// ds_read_b64_tr_b8 -- lane i of a 16-lane group gets column i of an 8-row x 16-byte block, lane l
// supplying row l / 2, bytes 8 (l % 2).. -- and widened to bf16 (exact: |code| <= 127); dW = unit *
// sum dy * code, the unit applied once in the epilogue.
// DIR (1x1, stride 1, pad 0: the gathered row of pixel m is x's row m): B rows addressed directly, no
// coordinate divisions. Both operands are DMA'd through buffer descriptors (a masked lane's offset is past
// the buffer: the hardware returns zeros), so a DMA is one v_cndmask, not an exec-masked pointer select.
template <int BMK, int NBUF, int BNC = 256, int XF = 0, int I8X = 0, int DIR = 0>
__global__ __launch_bounds__(BNC * 2, BNC == 256 ? 1 : 2) void wgrad_big_kernel(WgradArgs p) {
  static_assert(!(XF && I8X), "int8 input: no input transform");
  constexpr int CE = I8X ? 16 : 8, BKM = 64, XES = I8X ? 1 : 2;  // B chunk channels, B bytes per element
  constexpr int NWC = BNC / 64, NW = 2 * NWC;              // waves along the columns, waves
  constexpr int A_CPR = BMK / 8, B_CPR = BNC * XES / 16;  // 16-byte chunks per LDS row
  constexpr int A_RPI = 64 / A_CPR, B_RPI = 64 / B_CPR;  // rows per 1 KiB DMA instruction
  constexpr int AR = BKM / A_RPI / NW, BR = BKM / B_RPI / NW;  // DMA instructions per wave per M-tile
  constexpr int LPT = AR + BR;
  constexpr int MI = BMK / 32, NI = 4;
  constexpr int A_SZ = BKM * A_CPR, B_SZ = BKM * B_CPR;  // chunks
  constexpr int kStage = A_SZ + B_SZ;
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * kStage];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWC, wn = wid % NWC;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_split = p.nct * p.nkt;
  const int zs = lid / per_split;
  const int rem0 = lid - zs * per_split;
  const int kt = rem0 / p.nct;
  const int n0 = (rem0 - kt * p.nct) * BNC;
  const int k0 = kt * BMK;
  const int mbeg = zs * p.m_per_split;
  const int mend = min(p.M, mbeg + p.m_per_split);
  if (mbeg >= mend) return;

  // per-lane DMA rows (fixed within an M-tile) and source chunks
  int a_row[AR], a_col[AR];
#pragma unroll
  for (int j = 0; j < AR; ++j) {
    a_row[j] = (wid * AR + j) * A_RPI + lane / A_CPR;
    const int slot = lane % A_CPR;
    const int k = k0 + 8 * (slot ^ (swz_tr(a_row[j]) & (A_CPR - 1)));
    a_col[j] = k < p.ldy ? k : -1;
  }
  int b_row[BR], b_h[BR], b_w[BR], b_ch[BR];
#pragma unroll
  for (int j = 0; j < BR; ++j) {
    b_row[j] = (wid * BR + j) * B_RPI + lane / B_CPR;
    const int slot = lane % B_CPR;
    const int col = n0 + CE * (slot ^ ((I8X ? swz_tr8(b_row[j]) : swz_tr(b_row[j])) & (B_CPR - 1)));
    if (col < p.ncol_load && p.p4) {  // chunk = taps (r, s), (r, s + 1) of the padded image
      b_ch[j] = 0;
      b_h[j] = col >> 5;
      b_w[j] = (col >> 2) & 7;
    } else if (col < p.ncol_load) {
      const int tap = fdiv(col, p.fdC);
      b_ch[j] = col - tap * p.C;
      const int r = fdiv(tap, p.fdS);
      b_h[j] = r - p.ph;
      b_w[j] = tap - r * p.S - p.pw;
    } else {
      b_ch[j] = -1;
      b_h[j] = b_w[j] = 0;
    }
  }
  const v4i rs_dy = make_rsrc(p.dy, (uint32_t)p.dy_bytes);
  const v4i rs_x = make_rsrc(p.x, (uint32_t)p.x_bytes);
  const uint32_t lds_a = __builtin_amdgcn_readfirstlane(lds_addr(smem) + wid * AR * 1024);  // this wave's pieces
  const uint32_t lds_b = __builtin_amdgcn_readfirstlane(lds_addr(smem) + A_SZ * 16 + wid * BR * 1024);

  // branch-free (selects only), 32-bit byte offsets (both tensors < 4 GiB, host-checked), so the
  // compiler can interleave it with the MFMAs of the slab it is placed between
  auto issue = [&](int mb, int buf) __attribute__((always_inline)) {
    const uint32_t la = buf * (kStage * 16);
#pragma unroll
    for (int j = 0; j < AR; ++j) {
      const int m = mb + a_row[j];
      const bool ok = a_col[j] >= 0 && m < mend;
      dma16_asm(rs_dy, lds_a + la + j * 1024, ok ? (uint32_t)(m * p.ldy + a_col[j]) * 2u : kOob);
    }
#pragma unroll
    for (int j = 0; j < BR; ++j) {
      const int m = mb + b_row[j];
      if constexpr (DIR) {
        const bool ok = b_ch[j] >= 0 && m < mend;
        dma16_asm(rs_x, lds_b + la + j * 1024, ok ? (uint32_t)(m * p.C + b_ch[j]) * (uint32_t)XES : kOob);
      } else {
        const int n = fdiv(m, p.fdPQ);
        const int rem = m - n * p.P * p.Q;
        const int pp = fdiv(rem, p.fdQ);
        const int qq = rem - pp * p.Q;
        const int hin = pp * p.sh + b_h[j];
        const int win = qq * p.sw + b_w[j];
        const bool ok = b_ch[j] >= 0 && m < mend && (unsigned)hin < (unsigned)p.H && (unsigned)win < (unsigned)p.W;
        dma16_asm(rs_x, lds_b + la + j * 1024,
                  ok ? (uint32_t)(((n * p.H + hin) * p.W + win) * p.C + b_ch[j]) * (uint32_t)XES : kOob);
      }
    }
  };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float xsc[XF ? NI : 1], xsh[XF ? NI : 1];
  if constexpr (XF) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = n0 + wn * 64 + j * 16 + (lane & 15);
      xsc[j] = col < p.C ? p.in_sc[col] : 0.f;
      xsh[j] = col < p.C ? p.in_sh[col] : 0.f;
    }
  }

  auto compute = [&](int buf, int slab) __attribute__((always_inline)) {
    const char* Ab = reinterpret_cast<const char*>(smem + buf * kStage);
    const char* Bb = Ab + A_SZ * 16;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    {
      v8s af[MI], bfv[NI];
      if constexpr (I8X) {  // rows 8 g .. 8 g + 7 of the slab in one transposed byte read per fragment
        const int row = slab * 32 + 8 * g + (li >> 1);
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cb = wn * 64 + j * 16 + 8 * (li & 1);  // byte column
          const int byte = row * (B_CPR * 16) + (((cb >> 4) ^ (swz_tr8(row) & (B_CPR - 1))) << 4) + (cb & 15);
          const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(Bb + byte));
          bfv[j] = i8x8_to_bf16(v);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = slab * 32 + 8 * g + 4 * h + q;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if constexpr (I8X) break;
          const int col = wn * 64 + j * 16 + 4 * pp;
          const int byte = row * (B_CPR * 16) + ((((col * 2) >> 4) ^ (swz_tr(row) & (B_CPR - 1))) << 4) + ((col * 2) & 15);
          v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(Bb + byte));
#pragma unroll
          for (int e = 0; e < 4; ++e) bfv[j][4 * h + e] = v[e];
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int col = wm * (BMK / 2) + i * 16 + 4 * pp;
          const int byte = row * (A_CPR * 16) + ((((col * 2) >> 4) ^ (swz_tr(row) & (A_CPR - 1))) << 4) + ((col * 2) & 15);
          v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(Ab + byte));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][4 * h + e] = v[e];
        }
      }
      if constexpr (XF) {
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            bfv[j][e] = (short)f2bf(fmaxf(fmaf(bf2f((bf16_t)bfv[j][e]), xsc[j], xsh[j]), 0.f));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nstage = (mend - mbeg + BKM - 1) / BKM;
  // diagnostic build only (rn_set_tuning 6, bit mask; wrong results): 1 no dW epilogue, 2 no DMAs inside
  // the loop (the prologue's buffers are re-read), 4 no M-tile waits / barriers
  const int diag = kRnDiag ? p.diag_noepi : 0;
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(mbeg + s * BKM, s);
  for (int t = 0; t < nstage; ++t) {
    if (!(diag & 4)) {
      if (NBUF == 3) wait_vmcnt<LPT>();  // the later M-tile's DMAs (real or past the range) may stay in flight
      else wait_vmcnt<0>();
      __syncthreads();
    }
    compute(t % NBUF, 0);
    // unconditional (past the range every lane reads the zero chunk into a buffer nobody reads):
    // no branch, so the address arithmetic can interleave with slab 0's MFMAs
    if (!(diag & 2)) issue(mbeg + (t + NBUF - 1) * BKM, (t + NBUF - 1) % NBUF);
    compute(t % NBUF, 1);
  }
  wait_vmcnt<0>();

  // D[row = k][col] -> fp32 atomic add into dw (dense, unpadded: ldw = ncol); padded channels (the
  // stem's 3 of 8) keep c < creal
  if (kRnDiag && (diag & 1)) {  // keep the accumulators live without touching memory
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 12345.678f) p.dw[0] = s;
    return;
  }
  if constexpr (I8X) {  // dW = unit * sum dy * code
    const float u = *p.xunit;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] *= u;
  }
  const bool padded = p.creal != p.C;
  if (p.slab && !padded) {
    // this split's partial tile, staged through LDS (the operand buffers are free now) so that each store
    // instruction writes whole 256-byte rows (16 lanes x 16 bytes) instead of four 64-byte segments: per
    // wave SR rows x 64 columns at a time (64 rows: 8 waves x 16 KB = the 128 KB of the two 256x256
    // buffers; 32 where the int8-codes form's smaller buffers hold less). Column block j of staged row r
    // sits at block j ^ ((r >> 2) & 3): the two 32-lane halves of a b32 write (rows r, r + 4) and the
    // 16-lane groups of a b128 read (rows r, r + 1) meet no bank twice.
    float* dst = p.slab + (int64_t)zs * p.K * p.ldw;
    constexpr int SR = NBUF * kStage * 16 >= NW * 64 * 64 * 4 ? 64 : 32;
    static_assert(NW * SR * 64 * 4 <= NBUF * kStage * 16, "staging fits the operand buffers");
    constexpr int IR = SR / 16;                        // accumulator rows i per round
    constexpr int ROUNDS = (MI + IR - 1) / IR;
    float* stg = reinterpret_cast<float*>(smem) + wid * (SR * 64);
    __syncthreads();  // every wave is done reading the last M-tile's operands
#pragma unroll
    for (int hh = 0; hh < ROUNDS; ++hh) {
#pragma unroll
      for (int i = 0; i < IR; ++i) {
        if (hh * IR + i >= MI) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = i * 16 + (lane >> 4) * 4 + e;
#pragma unroll
          for (int j = 0; j < NI; ++j) stg[r * 64 + ((j ^ ((r >> 2) & 3)) << 4) + (lane & 15)] = acc[hh * IR + i][j][e];
        }
      }
      const int rows = (MI - hh * IR >= IR ? IR : MI - hh * IR) * 16;
#pragma unroll
      for (int t = 0; t < SR / 4; ++t) {
        const int r = t * 4 + (lane >> 4);
        if (r >= rows) break;
        const int c4 = (lane & 15) * 4;  // columns c4 .. c4 + 3 of the wave's 64
        const float4 v = *reinterpret_cast<const float4*>(stg + r * 64 + (((c4 >> 4) ^ ((r >> 2) & 3)) << 4) + (c4 & 15));
        const int k = k0 + wm * (BMK / 2) + hh * SR + r;
        const int col = n0 + wn * 64 + c4;
        if (k < p.K && col < p.ncol) *reinterpret_cast<float4*>(dst + (int64_t)k * p.ldw + col) = v;
      }
    }
    return;
  }
  // (padded channels: the slab, in the deterministic mode, takes the same compacted indices)
  float* const pdst = p.slab ? p.slab + (int64_t)zs * p.K * p.ldw : p.dw;
  auto put = [&](int64_t i, float v) __attribute__((always_inline)) {
    if (p.slab) pdst[i] = v;
    else atomicAdd(pdst + i, v);
  };
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + wm * (BMK / 2) + i * 16 + (lane >> 4) * 4 + e;
      if (k >= p.K) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wn * 64 + j * 16 + (lane & 15);
        if (!padded) {
          if (col < p.ncol) atomicAdd(p.dw + (int64_t)k * p.ldw + col, acc[i][j][e]);
        } else if (p.p4) {  // column (r*8 + s)*4 + c of the padded NHWC4 image
          const int c = col & 3, s = (col >> 2) & 7, r = col >> 5;
          if (c < p.creal && s < p.S && r < p.R) put((int64_t)k * p.ldw + (r * p.S + s) * p.creal + c, acc[i][j][e]);
        } else if (col < p.ncol_load) {
          const int tap = fdiv(col, p.fdC);
          const int c = col - tap * p.C;
          if (c < p.creal) put((int64_t)k * p.ldw + tap * p.creal + c, acc[i][j][e]);
        }
      }
    }
}

// ------------------------------------------------------------------------------ wgrad, image bands
// The weight gradient of a dense 3x3 / stride-1 / pad-1 convolution (the conv2 of every ResNet-50
// bottleneck unit but a stage's first, symbol/resnet.py:19-21): dW[k][tap][c] = sum_m dy[m][k] *
// x[m + tap shift][c]. A workgroup keeps a KS x 9 x CS slice of dW (channel slices: blockIdx.y over the
// input channels, blockIdx.z over the output channels) in its accumulators for all of its images,
// which it walks in bands of R output rows: per band the R dy rows and the R + 2 x rows they read are
// staged once (LDS-DMA) and every tap multiplies the same LDS image at a shifted row. Both images use
// a row stride of WP pixels with the x pixel (ih, iw) at column iw + 1: columns 0 and W + 1.. of x
// and W.. of dy are zero, so the shift r * WP + s of a dy pixel never needs an in-image test (dy is
// zero where a shifted read wraps). Each operand is read from HBM once per slice of the other (stage 1:
// the whole 64 x 576 dW in one workgroup, once); the tiled kernels gathered x per tap and column tile
// and ran at 6x these layers' memory time. 8 waves, wave (wk, wc) owns KB_W x CB_W 16-channel block
// pairs over all 9 taps (18 accumulators). Each workgroup stores its partial dW slice into the slab
// [split][K][9][C]; the split reduction pass sums them (deterministic order).
// The stream weight-gradient kernel's LDS swizzle: swz_tr, except for 8-chunk (128-byte, 64-channel) rows.
// (The image-band weight gradient keeps swz_tr: this swizzle made its LDS conflict-free there too, 0.500 ->
// 0.000, but measured 1.9 % slower in isolation and neutral in-step -- round 5, profiles/r05/ab/dband_swz --
// so it was reverted in round 6: that kernel is not LDS-bound.) A transposed
// 64-bit read's 32-lane group covers rows 8 g + 4 h + q (g = 0, 1; q = 0..3) at two chunks each; with
// 128-byte rows a row's bank half is row & 1, and swz_tr & 7 = 2 q drops g, so rows r and r + 8 hit the
// same banks (2-way: PMC 0.288 of the kernel's LDS cycles were conflicts on ResNet-50's 64-channel
// layers, profiles/r04/pmc_summary_resnet50_final.txt). Here the chunk pair of a row is 2 ((q >> 1) | 2 g):
// with q & 1 picking the bank half, the 8 rows x 2 chunks cover 16 distinct 16-byte bank groups.
__device__ __forceinline__ int swz_st(int row, int cpr) {
  return cpr == 8 ? 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) : swz_tr(row);
}
struct DbArgs {
  const bf16_t* x;   // [N][H][W][C]
  const bf16_t* dy;  // [N][H][W][K]
  float* slab;       // [split][K][9 * C]
  const float* in_sc;  // (XF) the producing BatchNorm's scale / shift: x := relu(x * sc + sh) on load
  const float* in_sh;
  int N, H, W, C, K, ipw;
};
template <int CS, int KS, int WP, int R>
struct DbShape {
  static constexpr int XCPR = CS / 8, DCPR = KS / 8;   // 16-byte chunks per pixel (x, dy slices)
  static constexpr int XPPI = 64 / XCPR, DPPI = 64 / DCPR;  // pixels per 1 KiB DMA instruction
  static constexpr int XPIX = (R + 2) * WP + 8;        // x rows oh0-1..oh0+R + a zero slack
  static constexpr int XINS = (R + 2) * WP / XPPI, DINS = R * WP / DPPI;
  static constexpr int INS = XINS + DINS, LPTM = (INS + 7) / 8;  // DMA instructions per band; per wave (max)
  static constexpr int XBYTES = XPIX * XCPR * 16;
  static constexpr int BUF = XPIX * XCPR + R * WP * DCPR;  // 16-byte chunks per band buffer
  static constexpr int CB = CS / 16, KB = KS / 16;
  static constexpr int WC = CB >= 8 ? 8 : CB, WK = 8 / WC;
  static constexpr int CB_W = CB / WC, KB_W = KB / WK;
  static_assert(CB_W * WC == CB && KB_W * WK == KB && CB_W * KB_W <= 2 && (R * WP) % 32 == 0 &&
                XPPI >= 1 && DPPI >= 1 && (R * WP) % DPPI == 0, "dense band shape");
};
// XF: the producing BatchNorm+ReLU (act2 = relu(bn2(conv1 out)), symbol/resnet.py:19-21) applied to
// the staged x image in place -- each thread rewrites the chunks its own DMAs landed, between its
// vmcnt wait and the band's barrier, max(x * sc + sh, 0) rounded to bf16 as bn_apply_kernel stores
// it; the chunks the DMA zero-filled (padding columns, rows outside the image) stay zero, as the conv
// pads the BN+ReLU output -- so act2 is never written (the forward applies it on load too).
template <int CS, int KS, int WP, int R, int NBUF, int XF = 0>
__global__ __launch_bounds__(512, 1) void wgrad_dband_kernel(DbArgs p) {
  using S = DbShape<CS, KS, WP, R>;
  constexpr int XCPR = S::XCPR, DCPR = S::DCPR, KB_W = S::KB_W, CB_W = S::CB_W;
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * S::BUF];
  __shared__ __attribute__((aligned(16))) float xtab[XF ? 2 * CS : 1];  // (XF) scale, shift of the slice
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n_first = blockIdx.x * p.ipw;
  const int n_end = min(p.N, n_first + p.ipw);
  const int bpi = (p.H + R - 1) / R;
  const int nb = (n_end - n_first) * bpi;
  const int c0 = blockIdx.y * CS, k0 = blockIdx.z * KS;  // the channel slices
  for (int i = tid; i < NBUF * 8 * XCPR; i += 512)
    smem[(i / (8 * XCPR)) * S::BUF + (R + 2) * WP * XCPR + i % (8 * XCPR)] = make_uint4(0, 0, 0, 0);
  if constexpr (XF) {
    for (int i = tid; i < CS; i += 512) {
      xtab[i] = p.in_sc[c0 + i];
      xtab[CS + i] = p.in_sh[c0 + i];
    }
  }
  uint32_t okb = 0;  // (XF) bit buf * LPTM + j: x piece j of the band in buffer buf holds image data
  // this wave's DMA pieces: w, w + 8, ... (x pieces first, then dy); lane = (pixel, LDS chunk slot), the
  // source chunk is the slot XOR the image's read swizzle
  const int cnt = (S::INS - wid + 7) / 8;
  int dr[S::LPTM], dc[S::LPTM], dch[S::LPTM];
  uint32_t dla[S::LPTM];
#pragma unroll
  for (int j = 0; j < S::LPTM; ++j) {
    const int piece = wid + 8 * j;
    const bool isx = piece < S::XINS;
    const int cpr = isx ? XCPR : DCPR;
    const int px = isx ? piece * S::XPPI + lane / XCPR : (piece - S::XINS) * S::DPPI + lane / DCPR;
    dr[j] = isx ? px / WP : -1 - px / WP;  // (dy pieces: -1 - row)
    dc[j] = px % WP;
    dch[j] = (isx ? c0 : k0) + 8 * ((lane % cpr) ^ (swz_tr(px) & (cpr - 1)));
    dla[j] = isx ? piece * 1024 : S::XBYTES + (piece - S::XINS) * 1024;
  }
  const char* zb = reinterpret_cast<const char*>(&g_zero_chunk);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  // band t's DMAs into buffer buf; past the last band (t >= nb) every lane reads the zero chunk, so each
  // wave issues the same count per band and the counted waits below hold to the end
  auto issue = [&](int t, int buf) __attribute__((always_inline)) {
    const bool live = t < nb;
    const int n = n_first + t / bpi, oh0 = R * (t % bpi);
    const uint32_t base = lds0 + buf * (S::BUF * 16);
    if constexpr (XF) okb &= ~(((1u << S::LPTM) - 1u) << (buf * S::LPTM));
#pragma unroll
    for (int j = 0; j < S::LPTM; ++j) {
      if (j >= cnt) break;  // (wave-uniform)
      const bf16_t* src;
      bool ok;
      if (dr[j] >= 0) {
        const int ih = oh0 - 1 + dr[j], iw = dc[j] - 1;
        ok = live && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        src = p.x + ((int64_t)(n * p.H + ih) * p.W + iw) * p.C + dch[j];
        if constexpr (XF) okb |= (uint32_t)ok << (buf * S::LPTM + j);
      } else {
        const int oh = oh0 - 1 - dr[j];
        ok = live && oh < p.H && dc[j] < p.W;
        src = p.dy + ((int64_t)(n * p.H + oh) * p.W + dc[j]) * p.K + dch[j];
      }
      dma16_global(ok ? (const void*)src : (const void*)zb, base + dla[j]);
    }
  };

  const int wk = wid / S::WC, wc = wid % S::WC;
  v4f acc[KB_W][CB_W][9];
#pragma unroll
  for (int i = 0; i < KB_W; ++i)
#pragma unroll
    for (int j = 0; j < CB_W; ++j)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[i][j][t] = v4f{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  // transposed 8-byte read of the 4 x 4 block at (pixel row, element column col) of an image with cpr
  // 16-byte chunks per pixel
  auto rd = [&](const char* img, int cpr, int row, int col) __attribute__((always_inline)) {
    const int byte = row * (cpr * 16) + ((((col * 2) >> 4) ^ (swz_tr(row) & (cpr - 1))) << 4) + ((col * 2) & 15);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + byte));
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* Xb = reinterpret_cast<const char*>(smem + buf * S::BUF);
    const char* Db = Xb + S::XBYTES;
#pragma unroll
    for (int ms = 0; ms < R * WP / 32; ++ms) {  // 32 dy pixels per step
      v8s af[KB_W], bfv[CB_W][9];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = ms * 32 + 8 * g + 4 * h + q;
#pragma unroll
        for (int i = 0; i < KB_W; ++i) {
          const v4s v = rd(Db, DCPR, row, (wk * KB_W + i) * 16 + 4 * pp);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][4 * h + e] = v[e];
        }
#pragma unroll
        for (int j = 0; j < CB_W; ++j)
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const v4s v = rd(Xb, XCPR, row + (t / 3) * WP + (t % 3), (wc * CB_W + j) * 16 + 4 * pp);
#pragma unroll
            for (int e = 0; e < 4; ++e) bfv[j][t][4 * h + e] = v[e];
          }
      }
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < CB_W; ++j)
#pragma unroll
          for (int i = 0; i < KB_W; ++i)
            acc[i][j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j][t], acc[i][j][t], 0, 0, 0);
    }
  };
  __syncthreads();  // (the slack zeros, the XF table)
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(s, s);
  for (int t = 0; t < nb; ++t) {
    // band t has landed once at most the DMAs of the NBUF - 2 bands issued after it are outstanding
    if (cnt == S::LPTM) wait_vmcnt<(NBUF - 2) * S::LPTM>();
    else wait_vmcnt<(NBUF - 2) * (S::LPTM - 1)>();
    if constexpr (XF) {  // this thread's landed x chunks of band t, transformed in place
      const int buf = t % NBUF;
#pragma unroll
      for (int j = 0; j < S::LPTM; ++j) {
        if (j >= cnt || dr[j] < 0) continue;  // (wave-uniform: the x pieces of this wave)
        uint4* cp = smem + buf * S::BUF + (dla[j] >> 4) + lane;
        const int cc = dch[j] - c0;
        float f[8], a[8], b[8];
        *reinterpret_cast<float4*>(a) = *reinterpret_cast<const float4*>(xtab + cc);
        *reinterpret_cast<float4*>(a + 4) = *reinterpret_cast<const float4*>(xtab + cc + 4);
        *reinterpret_cast<float4*>(b) = *reinterpret_cast<const float4*>(xtab + CS + cc);
        *reinterpret_cast<float4*>(b + 4) = *reinterpret_cast<const float4*>(xtab + CS + cc + 4);
        chunk_to_f(*cp, f, (const bf16_t*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], a[e], b[e]), 0.f);
        *cp = ((okb >> (buf * S::LPTM + j)) & 1u) ? f_to_chunk(f, (const bf16_t*)nullptr) : make_uint4(0, 0, 0, 0);
      }
    }
    __syncthreads();  // ... for every wave; and every wave is done with the buffer refilled next
    issue(t + NBUF - 1, (t + NBUF - 1) % NBUF);
    compute(t % NBUF);
  }
  wait_vmcnt<0>();  // (the zero-chunk DMAs past the last band land before the workgroup's LDS is released)
  // the workgroup's partial dW slice: slab[block][k][tap * C + c]
  float* dst = p.slab + (int64_t)blockIdx.x * p.K * 9 * p.C;
#pragma unroll
  for (int i = 0; i < KB_W; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + (wk * KB_W + i) * 16 + (lane >> 4) * 4 + e;
#pragma unroll
      for (int j = 0; j < CB_W; ++j)
#pragma unroll
        for (int t = 0; t < 9; ++t)
          dst[(int64_t)k * 9 * p.C + t * p.C + c0 + (wc * CB_W + j) * 16 + (lane & 15)] = acc[i][j][t][e];
    }
}

// The grouped form (ResNeXt's 3x3 / stride-1 convolutions, symbol/resnext.py:23-25, num_group = 32:
// 4 channels per group at C = 128 (stage 1, 56x56), 8 at C = 256 (stage 2, 28x28), 16 at C = 512
// (stage 3, 14x14)): the whole block-diagonal dW of a workgroup's images and channel slice in its
// accumulators. 16-channel block b of dy pairs with block b of x only (dW is zero across blocks), so
// wave w owns blocks w * BPW.. of the slice and every tap of them (9 * BPW accumulators); the MFMAs
// multiply whole 16 x 16 blocks and the epilogue keeps their group-diagonal G x G parts (with G < 16
// the MFMA work over the zero parts is the price of reading dy and x once: these layers are
// HBM-bound). Image rows of WP pixels (the x pixel (ih, iw) at column iw + 1), bands of R output
// rows; channel slices of CS channels (blockIdx.y; groups never straddle one) keep the band buffers
// double-buffered at C = 512. dW stored [K][3][3][G] into the slab. (The tiled grouped kernel re-read
// x per 64-column block and tap.)
struct GbArgs {
  const bf16_t* x;   // [N][H][W][C]
  const bf16_t* dy;  // [N][H][W][C]
  float* slab;       // [split][C][9 * G]
  int N, H, W, C, ipw;
};
template <int CS, int G, int WP, int R>
struct GbShape {
  static constexpr int CPR = CS / 8;                   // 16-byte chunks per pixel of the slice
  static constexpr int PPI = 64 / CPR;                 // pixels per 1 KiB DMA instruction
  static constexpr int XPIX = (R + 2) * WP + 8;        // x rows oh0-1..oh0+R + a zero slack
  static constexpr int XINS = (R + 2) * WP / PPI, DINS = R * WP / PPI;
  static constexpr int LPT = (XINS + DINS) / 8;        // DMA instructions per wave per band
  static constexpr int BUF = (XPIX + R * WP) * CPR;    // 16-byte chunks per band buffer
  static constexpr int BPW = CS / 16 / 8;              // 16-channel blocks per wave
  static_assert((XINS + DINS) % 8 == 0 && BPW >= 1 && (R * WP) % 32 == 0 && G <= 16, "grouped band shape");
};
template <int CS, int G, int WP, int R, int NBUF>
__global__ __launch_bounds__(512, 1) void wgrad_gband_kernel(GbArgs p) {
  using S = GbShape<CS, G, WP, R>;
  constexpr int CPR = S::CPR, PPI = S::PPI, BPW = S::BPW;
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * S::BUF];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n_first = blockIdx.x * p.ipw;
  const int n_end = min(p.N, n_first + p.ipw);
  const int bpi = (p.H + R - 1) / R;
  const int nb = (n_end - n_first) * bpi;
  const int c0 = blockIdx.y * CS;  // the channel slice
  for (int i = tid; i < NBUF * 8 * CPR; i += 512)
    smem[(i / (8 * CPR)) * S::BUF + (R + 2) * WP * CPR + i % (8 * CPR)] = make_uint4(0, 0, 0, 0);
  int dr[S::LPT], dc[S::LPT], dch[S::LPT];
  bool dx_[S::LPT];
#pragma unroll
  for (int j = 0; j < S::LPT; ++j) {
    const int piece = wid * S::LPT + j;
    dx_[j] = piece < S::XINS;
    const int px = (dx_[j] ? piece : piece - S::XINS) * PPI + lane / CPR;
    dr[j] = px / WP;
    dc[j] = px % WP;
    dch[j] = c0 + 8 * ((lane % CPR) ^ (swz_tr(px) & (CPR - 1)));
  }
  const char* zb = reinterpret_cast<const char*>(&g_zero_chunk);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  auto issue = [&](int t, int buf) __attribute__((always_inline)) {
    const int n = n_first + t / bpi, oh0 = R * (t % bpi);
    const uint32_t base = lds0 + buf * (S::BUF * 16);
#pragma unroll
    for (int j = 0; j < S::LPT; ++j) {
      const int piece = wid * S::LPT + j;
      const bf16_t* src;
      bool ok;
      uint32_t la;
      if (dx_[j]) {
        const int ih = oh0 - 1 + dr[j], iw = dc[j] - 1;
        ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        src = p.x + ((int64_t)(n * p.H + ih) * p.W + iw) * p.C + dch[j];
        la = base + piece * 1024;
      } else {
        const int oh = oh0 + dr[j];
        ok = oh < p.H && dc[j] < p.W;
        src = p.dy + ((int64_t)(n * p.H + oh) * p.W + dc[j]) * p.C + dch[j];
        la = base + S::XPIX * CPR * 16 + (piece - S::XINS) * 1024;
      }
      dma16_global(ok ? (const void*)src : (const void*)zb, la);
    }
  };
  v4f acc[BPW][9];
#pragma unroll
  for (int b = 0; b < BPW; ++b)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[b][t] = v4f{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  auto rd = [&](const char* img, int row, int col) __attribute__((always_inline)) {
    const int byte = row * (CPR * 16) + ((((col * 2) >> 4) ^ (swz_tr(row) & (CPR - 1))) << 4) + ((col * 2) & 15);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + byte));
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* Xb = reinterpret_cast<const char*>(smem + buf * S::BUF);
    const char* Db = Xb + S::XPIX * CPR * 16;
#pragma unroll
    for (int ms = 0; ms < R * WP / 32; ++ms) {
#pragma unroll
      for (int b = 0; b < BPW; ++b) {
        const int col = (wid * BPW + b) * 16 + 4 * pp;
        v8s af, bfv[9];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = ms * 32 + 8 * g + 4 * h + q;
          const v4s v = rd(Db, row, col);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[4 * h + e] = v[e];
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const v4s u = rd(Xb, row + (t / 3) * WP + (t % 3), col);
#pragma unroll
            for (int e = 0; e < 4; ++e) bfv[t][4 * h + e] = u[e];
          }
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[b][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[t], acc[b][t], 0, 0, 0);
      }
    }
  };
  __syncthreads();  // (the slack zeros)
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nb) issue(s, s);
  for (int t = 0; t < nb; ++t) {
    if (NBUF == 3 && t + 1 < nb) wait_vmcnt<S::LPT>();
    else wait_vmcnt<0>();
    __syncthreads();
    if (t + NBUF - 1 < nb) issue(t + NBUF - 1, (t + NBUF - 1) % NBUF);
    compute(t % NBUF);
  }
  // the group-diagonal G x G parts: slab[block][k][tap * G + c - group base]
  float* dst = p.slab + (int64_t)blockIdx.x * p.C * 9 * G;
#pragma unroll
  for (int b = 0; b < BPW; ++b)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = c0 + (wid * BPW + b) * 16 + (lane >> 4) * 4 + e;
      const int c = c0 + (wid * BPW + b) * 16 + (lane & 15);
      if (k / G != c / G) continue;
#pragma unroll
      for (int t = 0; t < 9; ++t) dst[(int64_t)k * 9 * G + t * G + c % G] = acc[b][t][e];
    }
}

// The weight gradient of a 1x1 / stride-1 convolution whose whole dW fits one workgroup's accumulators
// (K, C in {64, 128, 256}, K x C <= 32768: ResNet-50 / ResNeXt-50 stage 1's conv1 / conv3 / shortcut and
// stage 2's first conv1, symbol/resnet.py:17-31):
// dW = dy^T x over M = N*P*Q. Each workgroup streams ONE contiguous M range through NBUF LDS-DMA
// buffers of 64 rows (dy row: K channels, x row: C channels), so both operands are read from HBM once
// (the tiled kernels re-read one operand per output tile and ran at 3 TB/s, 2-3x this shape's memory
// time); the split partials go to the slab (wgrad_slab_reduce_kernel). XF: the producing
// BatchNorm+ReLU applied to the x fragments after their transposed read, as wgrad_big_kernel XF.
// 8 waves, wave (wk, wc) owns MI x NI 16x16 blocks of dW. I8X: x holds int8 codes, staged and read as
// wgrad_big_kernel I8X (the unit applied in the epilogue).
constexpr int stream_wk(int kb, int cb) {  // waves along K (of 8) minimizing the wave's A + B fragments
  int best = 0, cost = 1 << 30;
  for (int wk = 1; wk <= 8; wk *= 2) {
    const int wc = 8 / wk;
    if (kb % wk || cb % wc || (kb / wk) * (cb / wc) > 16) continue;
    if (kb / wk + cb / wc < cost) cost = kb / wk + cb / wc, best = wk;
  }
  return best;
}
template <int K, int C, int XF, int NBUF, int I8X = 0>
__global__ __launch_bounds__(512, 1) void wgrad_stream_kernel(WgradArgs p) {
  static_assert(!(XF && I8X), "int8 input: no input transform");
  constexpr int BKM = 64, XES = I8X ? 1 : 2, CEB = 16 / XES;   // B bytes per element, channels per chunk
  constexpr int A_CPR = K / 8, B_CPR = C / CEB;            // 16-byte chunks per LDS row
  constexpr int A_RPI = 64 / A_CPR, B_RPI = 64 / B_CPR;    // rows per 1 KiB DMA instruction
  constexpr int A_INS = BKM / A_RPI, B_INS = BKM / B_RPI;  // instructions per M-tile
  constexpr int TOT = A_INS + B_INS;
  // DMA pieces per wave: every wave issues LPT (the same count, for the vmcnt waits); past TOT a wave
  // re-issues the last piece (the same bytes to the same LDS chunk)
  constexpr int LPT = (TOT + 7) / 8;
  constexpr int KB = K / 16, CB = C / 16;
  constexpr int WK = stream_wk(KB, CB), WC = 8 / WK;  // (the split with the fewest fragment reads)
  constexpr int MI = KB / WK, NI = CB / WC;
  static_assert(WK > 0 && MI * WK == KB && NI * WC == CB && MI * NI <= 16, "wave tile");
  constexpr int A_SZ = BKM * A_CPR, B_SZ = BKM * B_CPR, kStage = A_SZ + B_SZ;
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * kStage];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid / WC, wc = wid % WC;
  const int zs = blockIdx.x;
  const int mbeg = zs * p.m_per_split;
  const int mend = min(p.M, mbeg + p.m_per_split);
  if (mbeg >= mend) return;
  // this wave's DMA pieces: piece j of the M-tile (A pieces first, then B)
  int d_row[LPT], d_col[LPT];
  bool d_isa[LPT];
#pragma unroll
  for (int j = 0; j < LPT; ++j) {
    const int piece = min(wid * LPT + j, TOT - 1);
    d_isa[j] = piece < A_INS;
    const int cpr = d_isa[j] ? A_CPR : B_CPR;
    const int row = d_isa[j] ? piece * A_RPI + lane / A_CPR : (piece - A_INS) * B_RPI + lane / B_CPR;
    d_row[j] = row;
    d_col[j] = d_isa[j] ? 8 * ((lane % cpr) ^ (swz_st(row, cpr) & (cpr - 1)))
                        : CEB * ((lane % cpr) ^ ((I8X ? swz_tr8(row) : swz_st(row, cpr)) & (cpr - 1)));
  }
  const char* __restrict__ dyb = reinterpret_cast<const char*>(p.dy);
  const char* __restrict__ xb = reinterpret_cast<const char*>(p.x);
  const char* zb = reinterpret_cast<const char*>(&g_zero_chunk);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  auto issue = [&](int mb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
      const int piece = min(wid * LPT + j, TOT - 1);
      const int m = mb + d_row[j];
      const bool ok = m < mend;
      const uint32_t off = d_isa[j] ? (uint32_t)(m * p.ldy + d_col[j]) * 2u : (uint32_t)(m * p.C + d_col[j]) * (uint32_t)XES;
      const char* src = d_isa[j] ? dyb + off : xb + off;
      const uint32_t la = lds0 + buf * (kStage * 16) +
                          (d_isa[j] ? piece * 1024 : A_SZ * 16 + (piece - A_INS) * 1024);
      dma16_global(ok ? (const void*)src : (const void*)zb, la);
    }
  };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float xsc[XF ? NI : 1], xsh[XF ? NI : 1];
  if constexpr (XF) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = (wc * NI + j) * 16 + (lane & 15);
      xsc[j] = p.in_sc[col];
      xsh[j] = p.in_sh[col];
    }
  }
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* Ab = reinterpret_cast<const char*>(smem + buf * kStage);
    const char* Bb = Ab + A_SZ * 16;
#pragma unroll
    for (int slab = 0; slab < 2; ++slab) {
      v8s af[MI], bfv[NI];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = slab * 32 + 8 * g + 4 * h + q;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int col = (wk * MI + i) * 16 + 4 * pp;
          const int byte = row * (A_CPR * 16) + ((((col * 2) >> 4) ^ (swz_st(row, A_CPR) & (A_CPR - 1))) << 4) + ((col * 2) & 15);
          const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(Ab + byte));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][4 * h + e] = v[e];
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if constexpr (I8X) break;
          const int col = (wc * NI + j) * 16 + 4 * pp;
          const int byte = row * (B_CPR * 16) + ((((col * 2) >> 4) ^ (swz_st(row, B_CPR) & (B_CPR - 1))) << 4) + ((col * 2) & 15);
          const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(Bb + byte));
#pragma unroll
          for (int e = 0; e < 4; ++e) bfv[j][4 * h + e] = v[e];
        }
      }
      if constexpr (I8X) {  // rows 8 g .. 8 g + 7 of the slab, one transposed byte read per fragment
        const int row = slab * 32 + 8 * g + (li >> 1);
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cb = (wc * NI + j) * 16 + 8 * (li & 1);
          const int byte = row * (B_CPR * 16) + (((cb >> 4) ^ (swz_tr8(row) & (B_CPR - 1))) << 4) + (cb & 15);
          const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(Bb + byte));
          bfv[j] = i8x8_to_bf16(v);
        }
      }
      if constexpr (XF) {  // (rows past the M range: their dy rows are zero)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            bfv[j][e] = (short)f2bf(fmaxf(fmaf(bf2f((bf16_t)bfv[j][e]), xsc[j], xsh[j]), 0.f));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nstage = (mend - mbeg + BKM - 1) / BKM;
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(mbeg + s * BKM, s);
  for (int t = 0; t < nstage; ++t) {
    if (NBUF == 3) wait_vmcnt<LPT>();  // the later M-tile's DMAs (real or past the range) may stay in flight
    else wait_vmcnt<0>();
    __syncthreads();
    issue(mbeg + (t + NBUF - 1) * BKM, (t + NBUF - 1) % NBUF);
    compute(t % NBUF);
  }
  wait_vmcnt<0>();
  const float us = I8X ? *p.xunit : 1.f;  // (I8X: dW = unit * sum dy * code)
  float* dst = p.slab + (int64_t)zs * K * C;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = (wk * MI + i) * 16 + (lane >> 4) * 4 + e;
#pragma unroll
      for (int j = 0; j < NI; ++j) dst[(int64_t)k * C + (wc * NI + j) * 16 + (lane & 15)] = I8X ? acc[i][j][e] * us : acc[i][j][e];
    }
}

// dw[i] += sum_z slab[z][i] (the split-M partial tiles of the weight-gradient kernels). A block takes 16
// float4 columns x 16 split groups: thread (g, c) sums splits g, g + 16, ... of column c in order, then
// the 16 group sums are added in group order (deterministic). (The first form gave each thread a whole
// column's splits, one block per 1,024 columns: ~36 blocks and a 256-long dependent chain per thread on
// a 64 x 576 dW -- ~2 TB/s.)
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(const float* __restrict__ slab, int nsplit,
                                                                int64_t n, float* __restrict__ dw) {
  if (n & 3) {  // (a split's slab not a whole number of 16-byte chunks: scalar, split order)
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
      float a = dw[i];
      for (int z = 0; z < nsplit; ++z) a += slab[(int64_t)z * n + i];
      dw[i] = a;
    }
    return;
  }
  const int64_t n4 = n / 4;
  const int cl = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int64_t col = blockIdx.x * 16 + cl;
  const float4* __restrict__ s4 = reinterpret_cast<const float4*>(slab);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < n4) {
    int z = sg;
    for (; z + 48 < nsplit; z += 64) {  // four loads in flight
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = s4[(int64_t)(z + 16 * u) * n4 + col];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
    for (; z < nsplit; z += 16) {
      const float4 v = s4[(int64_t)z * n4 + col];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  __shared__ float4 red[16][16];
  red[sg][cl] = a;
  __syncthreads();
  if (sg == 0 && col < n4) {
    float4 t = reinterpret_cast<const float4*>(dw)[col];
#pragma unroll
    for (int gi = 0; gi < 16; ++gi) {
      const float4 v = red[gi][cl];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    reinterpret_cast<float4*>(dw)[col] = t;
  }
}

// The same sum for at most 16 splits (the split-M grids sized for 45-50 % of the chip give 1-16): one
// thread per float4 column, every split's load in flight at once, added in split order onto dw --
// the value wgrad_slab_reduce_kernel stores (its 16 group sums are then the splits themselves and
// zeros; the one trailing + 0 reproduces its sign of a zero sum). The general kernel left 15/16 of its
// threads idle at these split counts.
__global__ __launch_bounds__(256) void wgrad_slab_reduce_few_kernel(const float* __restrict__ slab, int nsplit,
                                                                    int64_t n4, float* __restrict__ dw) {
  const int64_t col = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (col >= n4) return;
  const float4* __restrict__ s4 = reinterpret_cast<const float4*>(slab);
  float4 v[16];
#pragma unroll
  for (int z = 0; z < 16; ++z)
    if (z < nsplit) v[z] = s4[(int64_t)z * n4 + col];
  float4 t = reinterpret_cast<const float4*>(dw)[col];
  // each split as (0 + v), as the general kernel's group sum forms it: a -0 split adds +0, so the zero
  // sign of the result matches for every nsplit <= 16 (its empty groups then add +0 to an already
  // sign-normalised sum)
#pragma unroll
  for (int z = 0; z < 16; ++z)
    if (z < nsplit) {
      t.x += 0.f + v[z].x; t.y += 0.f + v[z].y; t.z += 0.f + v[z].z; t.w += 0.f + v[z].w;
    }
  reinterpret_cast<float4*>(dw)[col] = t;
}

// ------------------------------------------------------------------------------ helpers
template <typename T>
__global__ void pack_krsc_kernel(const float* __restrict__ wm, T* __restrict__ out, int K, int RS,
                                 int creal, int c) {
  const int64_t total = (int64_t)K * RS * c;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % c);
    const int64_t kt = i / c;  // k*RS + tap
    const float v = ci < creal ? wm[kt * creal + ci] : 0.f;
    out[i] = from_f<T>(v);
  }
}

template <typename T>
__global__ void pack_crsk_kernel(const float* __restrict__ wm, T* __restrict__ out, int K, int kpad,
                                 int RS, int creal, int c) {
  const int64_t total = (int64_t)c * RS * kpad;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % kpad);
    const int64_t ct = i / kpad;  // c*RS + tap
    const int tap = (int)(ct % RS);
    const int ci = (int)(ct / RS);
    float v = 0.f;
    if (k < K && ci < creal) v = wm[((int64_t)k * RS + tap) * creal + ci];
    out[i] = from_f<T>(v);
  }
}

// Grouped compute copy, block-diagonal over RN_GROUP_BLOCK-column blocks (see rn.h):
// out[col][tap][j], j < cblk: reduction index red = base(col's block) + j; nonzero only when
// red belongs to col's group. fwd (transpose 0): col = k, red = c. dgrad (1): col = c, red = k.
template <typename T>
__global__ void pack_group_kernel(const float* __restrict__ wm, T* __restrict__ out, int ncols, int RS,
                                  int cblk, int gcol, int gred, int cpg, int transpose) {
  const int64_t total = (int64_t)ncols * RS * cblk;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % cblk);
    const int64_t t = i / cblk;
    const int tap = (int)(t % RS);
    const int col = (int)(t / RS);
    const int n0 = col / RN_GROUP_BLOCK * RN_GROUP_BLOCK;
    const int red = (n0 / gcol) * gred + j;
    const int g = col / gcol;
    float v = 0.f;
    if (red / gred == g) {
      v = transpose ? wm[((int64_t)red * RS + tap) * cpg + (col - g * gcol)]
                    : wm[((int64_t)col * RS + tap) * cpg + (red - g * gred)];
    }
    out[i] = from_f<T>(v);
  }
}

// columns of one RN_GROUP_BLOCK block -> reduction channels it spans
inline int group_blk(int gcol, int gred) {
  return (gcol >= RN_GROUP_BLOCK ? 1 : RN_GROUP_BLOCK / gcol) * gred;
}

// ---- direct grouped 3x3 convolution: ResNeXt's 4 channels per group (symbol/resnext.py:23-25,
// num_group 32 at width 128; and the 8-per-group stride-2 forward). Block-diagonal MFMA tiles spend
// 15/16 of their products on zeros there; these layers need only 2 x 9 x G multiply-adds per byte, so
// VALU v_dot2_f32_bf16 (two bf16 products into fp32) on 16-byte channel chunks runs them near memory
// speed. Lane = (8-channel chunk, pixel lane): one wave instruction reads whole pixel rows
// (coalesced); a pixel lane computes PL consecutive output pixels of one row from the (PL-1)*ST+3
// input columns of each tap row (register reuse across the 3 horizontal taps and the PL pixels;
// interior windows skip the bounds tests); every chunk's weights sit in LDS, [chunk][tap][8 outputs]
// [G inputs] -- the compact compute copy (rn_conv_weight_pack). The data gradient of a stride-1 layer
// is the same kernel over dy with the group-transposed, tap-flipped copy (mode 1). (An MFMA variant --
// one wave per 16-channel chunk, tap pairs as the reduction, operands straight from global memory --
// measured 2x slower: its 32-byte-per-pixel loads touch 32 cache lines per wave instruction.)
typedef __bf16 __attribute__((ext_vector_type(2))) gd_bf2;
__device__ __forceinline__ float gd_dot(uint32_t x, uint32_t w, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(gd_bf2, x), __builtin_bit_cast(gd_bf2, w), acc, false);
}
struct GdArgs {
  const bf16_t* x;
  const bf16_t* w;
  bf16_t* y;
  const bf16_t* add;
  int H, W, C, P, Q, pad, lcpr, qb;  // input H x W, output P x Q, C channels (= 8 << lcpr), qb = ceil(Q / PL)
  uint32_t items;                    // N * P * qb pixel-lane work items
  FastDiv fdQB, fdP;
  // data gradient (RED), nullable: the BatchNorm-backward reduction of the gradient this layer completes,
  // as igemm_big_kernel's EPI 2 computes it (sum dz, sum dz*(x - mean), dz = dx * relu'(x sc + sh) on the
  // stored dx) -> bnred[block][C][2], one partial per workgroup
  float* bnred;
  const bf16_t* bn_x;
  const float *bn_mean, *bn_sc, *bn_sh;
  int bn_relu;
};
constexpr int kGdRedMaxC = 512;  // (gd_direct_shape: C / 8 divides 64)
// The table's index of channel ch: chunk k = ch / 8 starts at 16-byte slot 2 k + k / 2 + 2 (k / 4). The
// float4 reads of GdRed::add are ds_read_b128s whose lane groups are {0-3, 12-15, 20-27}, {4-11, 16-19,
// 28-31} and the same + 32 (MI355X_MICROARCH.md §LDS), lane l reading chunk l mod (C / 8); with the
// chunks 2 slots apart, groups put chunks 8 apart on one bank slot (0.58 of the stride-2 data gradient's
// LDS cycles were conflicts, profiles/r05/pmc_summary_resnext50.txt). This padding (found by search over
// C / 8 = 2 .. 64 chunks) gives every group 16 distinct slots for both halves of the chunk
__device__ __forceinline__ int gd_tab_idx(int ch) {
  const int k = ch >> 3;
  return 4 * (2 * k + (k >> 1) + 2 * (k >> 2)) + (ch & 7);
}
constexpr int kGdTab = 4 * (2 * 63 + 31 + 2 * 15 + 2);  // floats per table (64 chunks)
// LDS stride of one 8-channel chunk's weights, [tap][G] 16-byte rows plus one pad row: the lanes of a
// ds_read_b128 group read 16 different chunks at the same tap, and an unpadded stride of 9 G rows
// (144 / 288 dwords = 16 / 32 mod 64 banks) put 4 / 8 of them on the same banks (PMC: 0.78 / 0.85 of
// the LDS cycles were bank conflicts, profiles/r04/pmc_summary_resnext50.txt); 9 G + 1 rows = 148 / 292
// dwords step 20 / 36 banks, 5 c / 9 c mod 16 distinct over 16 chunks: conflict-free
template <int G>
constexpr int kGdWStride = 9 * G + 1;

// RED: one lane's stored output chunk into its BatchNorm-backward sums (channels chunk*8 .. +7). The
// per-channel mean / scale / shift sit in an LDS table (tab[3][C], loaded before the kernel's first
// barrier), not in registers: the direct kernels are latency bound and the 24 registers cost a wave
// per SIMD
struct GdRed {
  float s1[8], s2[8];
  __device__ __forceinline__ static void load_tab(const GdArgs& a, float* tab) {
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      tab[gd_tab_idx(c)] = a.bn_mean[c];
      tab[kGdTab + gd_tab_idx(c)] = a.bn_sc[c];
      tab[2 * kGdTab + gd_tab_idx(c)] = a.bn_sh[c];
    }
  }
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  }
  __device__ __forceinline__ void add(const GdArgs& a, const float* tab, int chunk, const uint4& out, int64_t off) {
    float g[8], xv[8], mu[8], sc[8], sh[8];
    chunk_to_f(out, g, (const bf16_t*)nullptr);
    chunk_to_f(*reinterpret_cast<const uint4*>(a.bn_x + off), xv, (const bf16_t*)nullptr);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ti = gd_tab_idx(chunk * 8);  // (a multiple of 4: 16-byte aligned)
      *reinterpret_cast<float4*>(mu + 4 * h) = reinterpret_cast<const float4*>(tab + ti)[h];
      *reinterpret_cast<float4*>(sc + 4 * h) = reinterpret_cast<const float4*>(tab + kGdTab + ti)[h];
      *reinterpret_cast<float4*>(sh + 4 * h) = reinterpret_cast<const float4*>(tab + 2 * kGdTab + ti)[h];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dz = (!a.bn_relu || fmaf(xv[e], sc[e], sh[e]) > 0.f) ? g[e] : 0.f;
      s1[e] += dz;
      s2[e] = fmaf(dz, xv[e] - mu[e], s2[e]);
    }
  }
  // lanes of one chunk (lane & (cpr - 1)) across the wave, then the block's waves through LDS, in a
  // fixed order: bnred[blockIdx.x][c][2]
  __device__ __forceinline__ void finish(const GdArgs& a, int chunk) {
    __shared__ float red[4][2][kGdRedMaxC];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int o = 1 << a.lcpr; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (lane < (1 << a.lcpr))
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wid][0][chunk * 8 + e] = s1[e];
        red[wid][1][chunk * 8 + e] = s2[e];
      }
    __syncthreads();
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      float t1 = 0.f, t2 = 0.f;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        t1 += red[w][0][c];
        t2 += red[w][1][c];
      }
      float* dst = a.bnred + ((int64_t)blockIdx.x * a.C + c) * 2;
      dst[0] = t1;
      dst[1] = t2;
    }
  }
};
template <int G, int ST, int PL, bool RED = false>
__global__ __launch_bounds__(256) void grouped_direct_kernel(GdArgs a) {
  extern __shared__ uint4 gd_w[];
  __shared__ __attribute__((aligned(16))) float gd_tab[RED ? 3 * kGdTab : 4];
  const int nw16 = a.C * 9 * G * 2 / 16;
  for (int i = threadIdx.x; i < nw16; i += blockDim.x)
    gd_w[i / (9 * G) * kGdWStride<G> + i % (9 * G)] = reinterpret_cast<const uint4*>(a.w)[i];
  if constexpr (RED) GdRed::load_tab(a, gd_tab);
  __syncthreads();
  constexpr int NC = (PL - 1) * ST + 3;
  const int lane = threadIdx.x & 63;
  const int chunk = lane & ((1 << a.lcpr) - 1), pl = lane >> a.lcpr;
  const int plw = 64 >> a.lcpr;
  const uint4* wc = gd_w + chunk * kGdWStride<G>;
  GdRed rd;
  if constexpr (RED) rd.init();
  const uint32_t step = gridDim.x * (blockDim.x >> 6) * plw;
  const int64_t cstep = a.C;
  for (uint32_t it = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * plw + pl; it < a.items; it += step) {
    const uint32_t t = fdiv(it, a.fdQB);
    const int q0 = (int)(it - t * a.qb) * PL;
    const uint32_t n = fdiv(t, a.fdP);
    const int p = (int)(t - n * a.P);
    const int w0 = q0 * ST - a.pad;
    const bool inner_w = w0 >= 0 && w0 + NC <= a.W;
    float acc[PL][8];
#pragma unroll
    for (int j = 0; j < PL; ++j)
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[j][o] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = p * ST - a.pad + r;
      if (h < 0 || h >= a.H) continue;
      const bf16_t* xrow = a.x + ((int64_t)(n * a.H + h) * a.W + w0) * cstep + chunk * 8;
      uint4 xc[NC];
      if (inner_w) {
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) xc[ci] = *reinterpret_cast<const uint4*>(xrow + ci * cstep);
      } else {
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
          const int w = w0 + ci;
          xc[ci] = (w >= 0 && w < a.W) ? *reinterpret_cast<const uint4*>(xrow + ci * cstep) : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int s_ = 0; s_ < 3; ++s_) {
        uint4 wv[G];
#pragma unroll
        for (int u = 0; u < G; ++u) wv[u] = wc[(r * 3 + s_) * G + u];
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(wv);  // pair jj of output o: wp[o * G / 2 + jj]
#pragma unroll
        for (int j = 0; j < PL; ++j) {
          const uint4 xv = xc[j * ST + s_];
          const uint32_t xp[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
          for (int o = 0; o < 8; ++o) {
            const int gb = G == 4 ? (o >> 2) * 2 : 0;  // first input pair of output o's group in the chunk
#pragma unroll
            for (int jj = 0; jj < G / 2; ++jj) acc[j][o] = gd_dot(xp[gb + jj], wp[o * (G / 2) + jj], acc[j][o]);
          }
        }
      }
    }
    const int64_t obase = ((int64_t)(n * a.P + p) * a.Q + q0) * cstep + chunk * 8;
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      if (q0 + j >= a.Q) break;
      const int64_t off = obase + j * cstep;
      if (a.add) {
        float f[8];
        chunk_to_f(*reinterpret_cast<const uint4*>(a.add + off), f, (const bf16_t*)nullptr);
#pragma unroll
        for (int o = 0; o < 8; ++o) acc[j][o] += f[o];
      }
      const uint4 out = f_to_chunk(acc[j], (const bf16_t*)nullptr);
      *reinterpret_cast<uint4*>(a.y + off) = out;
      if constexpr (RED) rd.add(a, gd_tab, chunk, out, off);
    }
  }
  if constexpr (RED) rd.finish(a, chunk);
}
// The data gradient of a STRIDE-2 direct grouped layer (3x3, pad 1): dx[h][w] = sum over the taps
// with (h + 1 - r) and (w + 1 - s) even of dy[(h + 1 - r) / 2][(w + 1 - s) / 2] * w[tap] -- an even
// output row takes tap row 1, an odd one rows 0 and 2; likewise columns, so a pixel lane's PL output
// pixels (from an even w0) read the PL/2 + 1 dy columns w0/2 .. w0/2 + PL/2 of each tap row. Same
// compact copy as the stride-1 data gradient (mode 1: tap 8 - t holds tap t), same lane layout.
template <int G, int PL, bool RED = false>
__global__ __launch_bounds__(256) void grouped_dgrad_s2_kernel(GdArgs a) {
  extern __shared__ uint4 gd_w[];
  __shared__ __attribute__((aligned(16))) float gd_tab[RED ? 3 * kGdTab : 4];
  const int nw16 = a.C * 9 * G * 2 / 16;
  for (int i = threadIdx.x; i < nw16; i += blockDim.x)
    gd_w[i / (9 * G) * kGdWStride<G> + i % (9 * G)] = reinterpret_cast<const uint4*>(a.w)[i];
  if constexpr (RED) GdRed::load_tab(a, gd_tab);
  __syncthreads();
  constexpr int ND = PL / 2 + 1;  // dy columns per tap row
  const int lane = threadIdx.x & 63;
  const int chunk = lane & ((1 << a.lcpr) - 1), pl = lane >> a.lcpr;
  const int plw = 64 >> a.lcpr;
  const uint4* wc = gd_w + chunk * kGdWStride<G>;
  GdRed rd;
  if constexpr (RED) rd.init();
  const uint32_t step = gridDim.x * (blockDim.x >> 6) * plw;
  const int64_t cstep = a.C;
  for (uint32_t it = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * plw + pl; it < a.items; it += step) {
    const uint32_t t = fdiv(it, a.fdQB);
    const int w0 = (int)(it - t * a.qb) * PL;  // (even)
    const uint32_t n = fdiv(t, a.fdP);
    const int h = (int)(t - n * a.P);
    float acc[PL][8];
#pragma unroll
    for (int j = 0; j < PL; ++j)
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[j][o] = 0.f;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      // even h: tap row 1 (dy row h / 2); odd h: rows 0 and 2 (dy rows (h + 1) / 2, (h - 1) / 2)
      const bool odd = h & 1;
      if (!odd && rr == 1) continue;
      const int r = odd ? 2 * rr : 1;
      const int pr = (h + 1 - r) >> 1;
      if (pr < 0 || pr >= a.H) continue;
      const bf16_t* dyrow = a.x + ((int64_t)(n * a.H + pr) * a.W + (w0 >> 1)) * cstep + chunk * 8;
      uint4 dc[ND];
#pragma unroll
      for (int ci = 0; ci < ND; ++ci)
        dc[ci] = ((w0 >> 1) + ci < a.W) ? *reinterpret_cast<const uint4*>(dyrow + ci * cstep) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int s_ = 0; s_ < 3; ++s_) {
        uint4 wv[G];
#pragma unroll
        for (int u = 0; u < G; ++u) wv[u] = wc[(8 - (r * 3 + s_)) * G + u];
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(wv);
#pragma unroll
        for (int j = 0; j < PL; ++j) {
          // even j (even w): tap column 1, dy column j / 2; odd j: columns 0 and 2, dy (j + 1) / 2, (j - 1) / 2
          if ((j & 1) == 0 && s_ != 1) continue;
          if ((j & 1) == 1 && s_ == 1) continue;
          const int ci = (j & 1) == 0 ? j / 2 : (s_ == 0 ? (j + 1) / 2 : (j - 1) / 2);
          const uint4 xv = dc[ci];
          const uint32_t xp[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
          for (int o = 0; o < 8; ++o) {
            const int gb = G == 4 ? (o >> 2) * 2 : 0;
#pragma unroll
            for (int jj = 0; jj < G / 2; ++jj) acc[j][o] = gd_dot(xp[gb + jj], wp[o * (G / 2) + jj], acc[j][o]);
          }
        }
      }
    }
    const int64_t obase = ((int64_t)(n * a.P + h) * a.Q + w0) * cstep + chunk * 8;
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      if (w0 + j >= a.Q) break;
      const int64_t off = obase + j * cstep;
      if (a.add) {
        float f[8];
        chunk_to_f(*reinterpret_cast<const uint4*>(a.add + off), f, (const bf16_t*)nullptr);
#pragma unroll
        for (int o = 0; o < 8; ++o) acc[j][o] += f[o];
      }
      const uint4 out = f_to_chunk(acc[j], (const bf16_t*)nullptr);
      *reinterpret_cast<uint4*>(a.y + off) = out;
      if constexpr (RED) rd.add(a, gd_tab, chunk, out, off);
    }
  }
  if constexpr (RED) rd.finish(a, chunk);
}

// compact compute copies of a direct grouped convolution (9 taps, G = cpg = kpg channels per group):
// mode 0: out[k/8][tap][k%8][c'] = w[k][tap][c']; mode 1 (stride-1 data gradient): out[c/8][tap][c%8][k']
// = w[g*G + k'][8 - tap][c - g*G], g = c / G (the group's outputs for input c, taps flipped)
__global__ void pack_group_direct_kernel(const float* __restrict__ wm, bf16_t* __restrict__ out, int C, int G,
                                         int transpose) {
  const int total = C * 9 * G;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int u = i % G, t = i / G;
    const int o = t % 8, t2 = t / 8;
    const int tap = t2 % 9, col = (t2 / 9) * 8 + o;
    const int g = col / G;
    const float v = transpose ? wm[((int64_t)(g * G + u) * 9 + (8 - tap)) * G + (col - g * G)]
                              : wm[((int64_t)col * 9 + tap) * G + u];
    out[i] = f2bf(v);
  }
}

// Many grouped compute copies in one launch (rn_conv_weight_pack_multi): blockIdx.y = copy, the
// items travel by value in the kernel argument. Element maps as pack_group_direct_kernel (direct)
// and pack_group_kernel (block-diagonal).
struct GpackItem {
  const float* wm;
  void* out;
  int64_t total;
  int direct, transpose, ncols, rs, cblk, gcol, gred, cpg;
};
constexpr int kGpackMax = 32;
struct GpackBatch {
  GpackItem it[kGpackMax];
};
template <typename T>
__global__ __launch_bounds__(256) void pack_group_multi_kernel(const GpackBatch b) {
  const GpackItem& p = b.it[blockIdx.y];
  T* __restrict__ out = reinterpret_cast<T*>(p.out);
  const float* __restrict__ wm = p.wm;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < p.total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (p.direct) {  // [C/8][9][8][G]
      const int G = p.cpg;
      const int u = (int)(i % G), t = (int)(i / G);
      const int o = t % 8, t2 = t / 8;
      const int tap = t2 % 9, col = (t2 / 9) * 8 + o;
      const int g = col / G;
      v = p.transpose ? wm[((int64_t)(g * G + u) * 9 + (8 - tap)) * G + (col - g * G)]
                      : wm[((int64_t)col * 9 + tap) * G + u];
    } else {  // [ncols][rs][cblk], block-diagonal
      const int j = (int)(i % p.cblk);
      const int64_t t = i / p.cblk;
      const int tap = (int)(t % p.rs);
      const int col = (int)(t / p.rs);
      const int n0 = col / RN_GROUP_BLOCK * RN_GROUP_BLOCK;
      const int red = (n0 / p.gcol) * p.gred + j;
      const int g = col / p.gcol;
      if (red / p.gred == g)
        v = p.transpose ? wm[((int64_t)red * p.rs + tap) * p.cpg + (col - g * p.gcol)]
                        : wm[((int64_t)col * p.rs + tap) * p.cpg + (red - g * p.gred)];
    }
    out[i] = from_f<T>(v);
  }
}

// thread per (row m, 16-byte output chunk): 8 (bf16) / 4 (f32) consecutive im2col columns
template <typename T>
__global__ __launch_bounds__(256) void im2col_nchw_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, T* __restrict__ cols, int N,
                                                          int C, int H, int W, int P, int Q, int R, int S, int sh,
                                                          int sw, int ph, int pw, int kc, FastDiv fdQ, FastDiv fdP,
                                                          FastDiv fdCH, const float* __restrict__ qthr, float qmax) {
  const float qt = qthr ? *qthr : 0.f;
  constexpr int CE = 16 / sizeof(T);
  const int cpr = kc / CE;
  const int64_t total = (int64_t)N * P * Q * cpr;
  const int kreal = R * S * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / cpr);
    const int ck = (int)(i - (int64_t)m * cpr);
    const int t2 = fdiv(m, fdQ);
    const int q = m - t2 * Q;
    const int n = fdiv(t2, fdP);
    const int pp = t2 - n * P;
    float v[CE];
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const int col = ck * CE + e;
      float val = 0.f;
      if (col < kreal) {
        const int tap = fdiv(col, fdCH);
        const int c = col - tap * C;
        const int r = tap / S, s = tap - (tap / S) * S;
        const int h = pp * sh - ph + r, w = q * sw - pw + s;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
          val = x[(((int64_t)n * C + c) * H + h) * W + w];
          if (scale) val = fmaf(val, scale[c], shift[c]);
          if (qthr) val = quant_value(val, qt, qmax, 1);  // conv0_data Quantization_int8
        }
      }
      v[e] = val;
    }
    reinterpret_cast<uint4*>(cols)[i] = f_to_chunk(v, (const T*)nullptr);
  }
}

// ---- quantized stem (symbol/resnet_int8.py:96-98: conv0 reads Quantization_int8(bn_data(x)))
// max |x*scale[c] + shift[c]| over the NCHW input
__global__ void stem_affine_absmax_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                          const float* __restrict__ shift, int64_t total, int C, int HW,
                                          float* __restrict__ out) {
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float v = x[i];
    if (scale) {
      const int c = (int)((i / HW) % C);
      v = fmaf(v, scale[c], shift[c]);
    }
    m = fmaxf(m, fabsf(v));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(m));
}
__global__ void stem_quant_state_kernel(float* __restrict__ curmax, float* minmax, int is_train, float decay,
                                        int first, float* __restrict__ thr) {
  *thr = quant_state_update(*curmax, minmax, 0, is_train, decay, first);
  *curmax = 0.f;  // the quantizers' shared-workspace invariant (rn_quant_int8_fwd): ws[0] left zero
}
// The activation STE zeroes the gradient where |v| >= t (clip_grad_quantization_int8.py:56-67).
// rn_stem_shift_grad sums the unmasked gradient; subtract the clipped elements' share:
// dbeta[c] -= dx[n,c,h,w] at every clipped (n,c,h,w), dx = sum_{k,r,s} w[k,r,s,c] dy[n,p,q,k].
__device__ __forceinline__ void load4f(const bf16_t* p, float* o) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  o[0] = bf2f((bf16_t)(u.x & 0xffffu));
  o[1] = bf2f((bf16_t)(u.x >> 16));
  o[2] = bf2f((bf16_t)(u.y & 0xffffu));
  o[3] = bf2f((bf16_t)(u.y >> 16));
}
__device__ __forceinline__ void load4f(const float* p, float* o) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x;
  o[1] = v.y;
  o[2] = v.z;
  o[3] = v.w;
}
struct ClipGeo {
  int N, C, H, W, P, Q, K, kpad, R, S, sh, sw, ph, pw;
  FastDiv fdHW, fdC, fdW, fdSH, fdSW;
};
template <typename T>
__global__ __launch_bounds__(256) void stem_clip_grad_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ thr, const T* __restrict__ dy,
                                                             const float* __restrict__ wq, float* __restrict__ dbeta,
                                                             const ClipGeo gm) {
  // A wave tests 256 consecutive input elements (a 16-byte load per lane), then takes the clipped ones
  // (ballot) four at a time: a 16-lane group per element, each lane 4 consecutive output channels k
  // (one 8-byte dy load per tap, the group reading the tap's whole 128-byte row; the weights from an
  // LDS copy laid out [c][r][s][k], one 16-byte read per tap), the index math per lane on the vector
  // unit. (The first form -- one element per wave, lanes over k, its index math and tap tests on the
  // scalar unit -- was bound by that unit, which a CU's four SIMDs share: ~700 scalar instructions per
  // clipped element, 0.96 ms at the bench's ~1.2 % clipped elements.) Image data saturates (pixel
  // value 255 IS the max), so a few 0.1 % of the elements clip.
  extern __shared__ __attribute__((aligned(16))) float wl[];
  __shared__ float wsum[4][8];
  const int C = gm.C, H = gm.H, W = gm.W, P = gm.P, Q = gm.Q, K = gm.K, R = gm.R, S = gm.S;
  const int RSK = R * S * K, nwl = C * RSK;
  for (int i = threadIdx.x; i < nwl; i += blockDim.x) {
    const int k = i % K, rest = i / K;
    const int s_ = rest % S, rr = rest / S;
    const int r = rr % R, c = rr / R;
    wl[i] = wq[((k * R + r) * S + s_) * C + c];
  }
  if (threadIdx.x < 32) wsum[threadIdx.x >> 3][threadIdx.x & 7] = 0.f;
  __syncthreads();
  const float t = *thr;
  const int HW = H * W, total = gm.N * C * HW;
  const int lane = threadIdx.x & 63, grp = lane >> 4, l4 = (lane & 15) * 4;
  const bool kok = l4 < K;
  auto gather4 = [&](int e) {  // e < 0: no element for this lane group
    float g = 0.f;
    int c = 0;
    if (e >= 0) {
      const int plane = (int)fdiv((uint32_t)e, gm.fdHW), hw = e - plane * HW;
      const int n = (int)fdiv((uint32_t)plane, gm.fdC);
      c = plane - n * C;
      const int h = (int)fdiv((uint32_t)hw, gm.fdW), w = hw - h * W;
      const int hq = (int)fdiv((uint32_t)(h + gm.ph), gm.fdSH), wq_ = (int)fdiv((uint32_t)(w + gm.pw), gm.fdSW);
      const int r0 = h + gm.ph - hq * gm.sh, s0 = w + gm.pw - wq_ * gm.sw;
      const T* dyn = dy + (int64_t)n * P * Q * gm.kpad + (kok ? l4 : 0);
      float dv[4][4][4];
      int wo[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int r = r0 + a * gm.sh, s_ = s0 + b * gm.sw;
          const int pp = hq - a, qq = wq_ - b;
          const bool ok = kok && r < R && s_ < S && pp >= 0 && qq >= 0 && pp < P && qq < Q;
          // unconditional load from a clamped (in-range) address, the value selected after it
          const int ppc = min(max(pp, 0), P - 1), qqc = min(max(qq, 0), Q - 1);
          load4f(dyn + (int64_t)(ppc * Q + qqc) * gm.kpad, dv[a][b]);
#pragma unroll
          for (int u = 0; u < 4; ++u) dv[a][b][u] = ok ? dv[a][b][u] : 0.f;
          wo[a][b] = ok ? ((c * R + r) * S + s_) * K + l4 : 0;
        }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const float4 wv = *reinterpret_cast<const float4*>(wl + wo[a][b]);
          g = fmaf(wv.x, dv[a][b][0], g);
          g = fmaf(wv.y, dv[a][b][1], g);
          g = fmaf(wv.z, dv[a][b][2], g);
          g = fmaf(wv.w, dv[a][b][3], g);
        }
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) g += __shfl_xor(g, off, 64);  // the group's 16 lanes
    if ((lane & 15) == 0 && e >= 0) atomicAdd(&wsum[threadIdx.x >> 6][c], -g);
  };
  auto clipped_at = [&](float xv, int e) {
    const int c = (e / HW) % C;
    const float v = scale ? fmaf(xv, scale[c], shift[c]) : xv;
    return !(v > -t && v < t);
  };
  // up to four set bits of the (wave-uniform) mask m, lowest first, to the four lane groups
  auto take4 = [&](uint64_t& m, int e0) {
    int eg = -1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (m) {
        const int b = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        if (grp == q) eg = e0 + b;
      }
    }
    return eg;
  };
  const int nv = total / 4;  // 16-byte chunks, then the tail
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  for (int base = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; base < nv; base += nwaves * 64) {
    const int i = base + lane;
    bool cl[4] = {false, false, false, false};
    if (i < nv) {
      const float4 v4 = reinterpret_cast<const float4*>(x)[i];
      cl[0] = clipped_at(v4.x, 4 * i);
      cl[1] = clipped_at(v4.y, 4 * i + 1);
      cl[2] = clipped_at(v4.z, 4 * i + 2);
      cl[3] = clipped_at(v4.w, 4 * i + 3);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t m = __ballot(cl[j]);
      while (m) {  // element of bit b: 4 * (base + b) + j
        const int b4 = take4(m, 0);
        gather4(b4 >= 0 ? 4 * (base + b4) + j : -1);
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // the last total % 4 elements: wave 0 of block 0
    const int e = 4 * nv + lane;
    uint64_t m = __ballot(e < total && clipped_at(x[e], e));
    while (m) gather4(take4(m, 4 * nv));
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const float v = wsum[0][threadIdx.x] + wsum[1][threadIdx.x] + wsum[2][threadIdx.x] + wsum[3][threadIdx.x];
    if (v != 0.f) atomicAdd(dbeta + threadIdx.x, v);
  }
}

// S[p][q][k] = sum_n dy[n][p][q][k]: thread per 16-byte chunk of one image (kpad is a multiple of
// the chunk), 8 images in flight per thread (a plain HBM-bound reduction over the batch)
template <typename T>
__global__ __launch_bounds__(256) void stem_sum_n_kernel(const T* __restrict__ dy, float* __restrict__ ws, int N,
                                                         int PQ, int kpad) {
  constexpr int CE = 16 / sizeof(T);
  const int64_t total = (int64_t)PQ * kpad;
  const int64_t nch = total / CE;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nch; i += (int64_t)gridDim.x * blockDim.x) {
    float acc[CE];
#pragma unroll
    for (int e = 0; e < CE; ++e) acc[e] = 0.f;
    const uint4* src = reinterpret_cast<const uint4*>(dy) + i;
    int n = 0;
    for (; n + 8 <= N; n += 8) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(n + u) * nch];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float f[CE];
        chunk_to_f(v[u], f, (const T*)nullptr);
#pragma unroll
        for (int e = 0; e < CE; ++e) acc[e] += f[e];
      }
    }
    for (; n < N; ++n) {
      float f[CE];
      chunk_to_f(src[(int64_t)n * nch], f, (const T*)nullptr);
#pragma unroll
      for (int e = 0; e < CE; ++e) acc[e] += f[e];
    }
#pragma unroll
    for (int e = 0; e < CE; ++e) ws[i * CE + e] = acc[e];
  }
}
// separable rectangle sums: Tq[p][s][k] = sum_{q in V(s)} S[p][q][k];
// G[k][r][s] = sum_{p in V(r)} Tq[p][s][k]   (V = output positions whose tap lands in-bounds)
__global__ void stem_colsum_kernel(const float* __restrict__ ws, float* __restrict__ tq, int K, int kpad, int S,
                                   int W, int P, int Q, int sw, int pw) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= P * S * K) return;
  const int k = idx % K;
  const int s = (idx / K) % S;
  const int pp = idx / (K * S);
  // the in-bounds output columns of tap s: 0 <= q*sw - pw + s < W (a contiguous range)
  const int qlo = max(0, (pw - s + sw - 1) / sw);  // (a negative numerator only gives values <= 0)
  const int qhi = W - 1 + pw - s < 0 ? -1 : min(Q - 1, (W - 1 + pw - s) / sw);
  const float* src = ws + (int64_t)pp * Q * kpad + k;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // independent chains: the loads overlap
  int q = qlo;
  for (; q + 3 <= qhi; q += 4) {
    a0 += src[(int64_t)q * kpad];
    a1 += src[(int64_t)(q + 1) * kpad];
    a2 += src[(int64_t)(q + 2) * kpad];
    a3 += src[(int64_t)(q + 3) * kpad];
  }
  for (; q <= qhi; ++q) a0 += src[(int64_t)q * kpad];
  tq[idx] = (a0 + a1) + (a2 + a3);
}
__global__ void stem_tap_sum_kernel(const float* __restrict__ tq, float* __restrict__ g, int K, int R, int S, int H,
                                    int P, int sh, int ph) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= K * R * S) return;
  const int k = idx / (R * S);
  const int tap = idx % (R * S);
  const int r = tap / S, s = tap % S;
  const int plo = max(0, (ph - r + sh - 1) / sh);
  const int phi = H - 1 + ph - r < 0 ? -1 : min(P - 1, (H - 1 + ph - r) / sh);
  const float* src = tq + (int64_t)s * K + k;
  const int64_t step = (int64_t)S * K;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int pp = plo;
  for (; pp + 3 <= phi; pp += 4) {
    a0 += src[pp * step];
    a1 += src[(pp + 1) * step];
    a2 += src[(pp + 2) * step];
    a3 += src[(pp + 3) * step];
  }
  for (; pp <= phi; ++pp) a0 += src[pp * step];
  g[idx] = (a0 + a1) + (a2 + a3);
}
__global__ void stem_shift_reduce_kernel(const float* __restrict__ g, const float* __restrict__ wm,
                                         float* __restrict__ dbeta, int K, int RS, int C) {
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int i = threadIdx.x; i < K * RS; i += blockDim.x) acc += g[i] * wm[(int64_t)i * C + c];
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dbeta[c] += red[0];
}

template <typename T, bool XF>
void launch_wgrad_tiles(int bmk, int bnc, dim3 grid, hipStream_t st, const WgradArgs& a) {
  if (bmk == 64 && bnc == 64) hipLaunchKernelGGL((wgrad_kernel<T, 64, 64, XF>), grid, dim3(256), 0, st, a);
  else if (bmk == 64) hipLaunchKernelGGL((wgrad_kernel<T, 64, 128, XF>), grid, dim3(256), 0, st, a);
  else if (bnc == 64) hipLaunchKernelGGL((wgrad_kernel<T, 128, 64, XF>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((wgrad_kernel<T, 128, 128, XF>), grid, dim3(256), 0, st, a);
}

int grid_for(int64_t total, int block = 256) {
  int64_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}
// wgrad_slab_reduce_kernel's grid: 16 float4 columns per block (the scalar path: a grid-stride loop)
int slab_reduce_blocks(int64_t n) {
  if (n & 3) return grid_for(n);
  return (int)std::max<int64_t>(1, (n / 4 + 15) / 16);
}
// dw[i] += sum_z slab[z][i]: the few-split kernel for <= 16 splits of whole 16-byte chunks (rn_set_tuning 25
// = 1: the general kernel always)
void launch_slab_reduce(const float* slab, int split, int64_t n, float* dw, hipStream_t st) {
  if (split <= 16 && (n & 3) == 0 && g_tune[RN_TUNE_SLAB_FEW] != 1)
    hipLaunchKernelGGL(wgrad_slab_reduce_few_kernel, dim3((unsigned)std::max<int64_t>(1, (n / 4 + 255) / 256)), dim3(256),
                       0, st, slab, split, n / 4, dw);
  else
    hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3(slab_reduce_blocks(n)), dim3(256), 0, st, slab, split, n, dw);
}

// Build igemm args for fwd (mode 0) or dgrad (mode 1).
// fwd : gathered = x (N,H,W,C), out = y (N,P,Q,K), B = w_krsc [K][R][S][C]
// dgrad: gathered = dy (N,P,Q,k_pad), out = dx (N,H,W,c), B = w_crsk [c][R][S][k_pad]
IgemmArgs make_igemm_args(const rn_conv_desc* d, int mode) {
  IgemmArgs a{};
  a.S = d->s;
  if (mode == 0) {
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c;
    a.P = d->p; a.Q = d->q; a.K = d->k; a.ldo = d->k_pad;
    a.wrow = d->r * d->s * d->c;
    a.rstep = 1; a.sstep = 1;
    a.hmul = d->stride_h; a.wmul = d->stride_w;
    a.hinc = 1; a.winc = 1;
    a.ostep_h = 1; a.ostep_w = 1;
    a.gcol = 1 << 30; a.gred = 0; a.cblk = a.C;
    if (d->groups > 1) {
      a.gcol = d->k / d->groups; a.gred = d->c / d->groups;
      a.cblk = group_blk(a.gcol, a.gred);
      a.wrow = d->r * d->s * a.cblk;
    }
    const int stage_elems = d->dtype == RN_BF16 ? 64 : 32;
    if (d->groups == 1 && d->c < stage_elems && (d->c & (d->c - 1)) == 0 && d->r * d->s > 1) {
      a.smallc = 1;
      a.lgc = __builtin_ctz(d->c);
      a.rs = d->r * d->s;
      a.fdS = make_fastdiv(d->s);
    }
    a.ncls = 1;
    IgemmCls& c = a.cls[0];
    c.a = 0; c.b = 0; c.Pc = d->p; c.Qc = d->q; c.r0 = 0; c.s0 = 0; c.nr = d->r; c.ns = d->s;
    c.hoff0 = 0; c.woff0 = 0; c.hb0 = -d->pad_h; c.wb0 = -d->pad_w;
    c.fdQ = make_fastdiv(c.Qc); c.fdPQ = make_fastdiv(c.Pc * c.Qc);
  } else {
    a.N = d->n; a.H = d->p; a.W = d->q; a.C = d->k_pad;
    a.P = d->h; a.Q = d->w; a.K = d->c; a.ldo = d->c;
    a.wrow = d->r * d->s * d->k_pad;
    a.rstep = d->stride_h; a.sstep = d->stride_w;
    a.hmul = 1; a.wmul = 1;
    a.hinc = -1; a.winc = -1;
    a.ostep_h = d->stride_h; a.ostep_w = d->stride_w;
    a.gcol = 1 << 30; a.gred = 0; a.cblk = a.C;
    if (d->groups > 1) {
      a.gcol = d->c / d->groups; a.gred = d->k / d->groups;
      a.cblk = group_blk(a.gcol, a.gred);
      a.wrow = d->r * d->s * a.cblk;
    }
    a.ncls = d->stride_h * d->stride_w;
    for (int z = 0; z < a.ncls; ++z) {
      IgemmCls& c = a.cls[z];
      c.a = z / d->stride_w; c.b = z % d->stride_w;
      c.Pc = (int)ceil_div(d->h - c.a, d->stride_h);
      c.Qc = (int)ceil_div(d->w - c.b, d->stride_w);
      if (c.Pc < 0) c.Pc = 0;
      if (c.Qc < 0) c.Qc = 0;
      c.r0 = (c.a + d->pad_h) % d->stride_h;
      c.s0 = (c.b + d->pad_w) % d->stride_w;
      c.nr = c.r0 < d->r ? (int)ceil_div(d->r - c.r0, d->stride_h) : 0;
      c.ns = c.s0 < d->s ? (int)ceil_div(d->s - c.s0, d->stride_w) : 0;
      c.hoff0 = (c.a + d->pad_h - c.r0) / d->stride_h;
      c.woff0 = (c.b + d->pad_w - c.s0) / d->stride_w;
      c.hb0 = 0; c.wb0 = 0;
      c.fdQ = make_fastdiv(c.Qc > 0 ? c.Qc : 1);
      c.fdPQ = make_fastdiv(c.Pc * c.Qc > 0 ? c.Pc * c.Qc : 1);
    }
  }
  return a;
}

// The 4-wave one-buffer 224x128 tile (igemm_big_kernel W4, two workgroups per CU) for these
// arguments? rn_set_tuning 11: 0 auto (forward 1x1, pad 0, >= 1024 tiles: the stage-1 conv3 / shortcut
// layers, 230 -> 215 us; since round 5 also the deeper ones -- stage-2 unit-1 conv1 163 -> 131 us,
// stage-3 unit-1 conv1 83 -> 77 us in isolation, ResNet-50 20.45 / 20.44 -> 20.42 / 20.40 ms per step;
// the data gradients and the grids under 1024 tiles measured no better or slower), 1 never,
// 2 every eligible 1x1 pad-0 layer, fwd and dgrad (tests), 3 the round-4 rule (one K-tile only).
bool w4_tile(const IgemmArgs& a) {
  const int mode = g_tune[RN_TUNE_IGEMM_W4];
  if (mode == 1 || g_tune[RN_TUNE_IGEMM_ROWS] == 1 || a.ncls != 1 || a.gred > 0 || a.smallc || a.bias || a.K <= 64)
    return false;
  const IgemmCls& c = a.cls[0];
  if (c.nr != 1 || c.ns != 1 || c.hoff0 != 0 || c.woff0 != 0 || c.hb0 != 0 || c.wb0 != 0) return false;
  if (a.in_sc && a.C > kXfMaxCW4) return false;
  if (mode == 2) return true;
  const int64_t tiles = ceil_div((int64_t)a.N * c.Pc * c.Qc, 224) * ceil_div(a.K, 128);
  if (mode == 3) return a.hinc > 0 && ceil_div(a.cblk, 64) == 1 && tiles >= 1024;  // (round-4 rule: one K-tile)
  return a.hinc > 0 && tiles >= 1024;
}

// Columns of the 256-row tile launch_igemm runs for these arguments (bf16 in and out), 0 for the
// 128-row kernel. rn_set_tuning 4: 0 auto, 1 off, 2 force 256x256, 3 force 256x128. Auto, from
// per-layer measurements over ResNet-50 (tools/conv_bench.py): 256x256 when the output has >= 256
// columns and the grid still has >= 192 tiles (one workgroup per CU; fewer leave too many CUs
// idle), else 256x128 when it has >= 128 columns, else the 128-row kernel.
int big_tile_cols(const IgemmArgs& a, int64_t xb, int64_t wb) {
  const int big = g_tune[RN_TUNE_IGEMM_BIG];
  int max_taps = 0;
  for (int z = 0; z < a.ncls; ++z) max_taps = std::max(max_taps, a.cls[z].nr * a.cls[z].ns);
  if (a.gred > 0) {  // grouped (ResNeXt): the 256x64 tile over one RN_GROUP_BLOCK column block, deep reductions
    // (rn_set_tuning 13 = 2: also the stride-2 data gradients, whose parity classes have <= 4 taps)
    const int nst = max_taps * (int)ceil_div(a.cblk, 64);
    const int min_nst = g_tune[RN_TUNE_IGEMM_GD] == 2 ? 4 : 8;
    return (big != 1 && big != 5 && RN_GROUP_BLOCK == 64 && !a.in_sc && !a.bias && !g_tune[RN_TUNE_DIAG_IGEMM_L1] &&
            xb < INT32_MAX && wb < INT32_MAX && max_taps <= 32 && nst >= min_nst) ? 64 : 0;
  }
  if (a.smallc)  // the stem (C = 8): the 256x64 tile in its small-C mode (rn_set_tuning 4 = 1 or 5: never)
    return (big != 1 && big != 5 && a.C == 8 && a.K <= 64 && !a.in_sc && !a.bias && !g_tune[RN_TUNE_DIAG_IGEMM_L1] &&
            xb < INT32_MAX && wb < INT32_MAX) ? 64 : 0;
  // the BN+ReLU input transform (in_sc) runs on the 224-row 128/256-column tiles, and on the 64-column
  // tile when C = 64 (its scale / shift in registers)
  const bool xf_ok = !a.in_sc || (a.K > 64 ? a.C <= kXfMaxC && g_tune[RN_TUNE_IGEMM_ROWS] != 1 : a.C == 64 && a.cblk == 64);
  const bool eligible = big != 1 && xf_ok && a.gred == 0 && !g_tune[RN_TUNE_DIAG_IGEMM_L1] &&
                        !a.bias && xb < INT32_MAX && wb < INT32_MAX && max_taps <= 32;
  if (!eligible) return 0;
  if (a.K <= 64) {  // 4-wave 256x64 tile where the reduction is deep (>= 8 K-tiles: the 3x3 layers);
                   // on the short 1x1 reductions the 128-row kernel measured faster (rn_set_tuning 4 = 5: never)
    const int nst = max_taps * (int)ceil_div(a.cblk, 64);
    return (big == 5 || nst < 8) ? 0 : 64;
  }
  if (big == 2) return 256;
  if (big == 3) return 128;
  if (w4_tile(a)) return 128;
  int64_t rows = 0;  // 256-row tiles over all parity classes
  for (int z = 0; z < a.ncls; ++z) rows += ceil_div((int64_t)a.N * a.cls[z].Pc * a.cls[z].Qc, 256);
  return (a.K >= 256 && rows * ceil_div(a.K, 256) >= 192) ? 256 : 128;
}

// Rows of the 256-row-family tile for `bn` columns: 224 (16x16 MFMAs) unless rn_set_tuning 9 = 1,
// or the 64-column tile. The BatchNorm epilogue partials cover one wave row (half the tile).
int big_tile_rows(int bn) { return (bn >= 128 && g_tune[RN_TUNE_IGEMM_ROWS] != 1) ? 224 : 256; }

// rows per BatchNorm partial block of the conv kernel these arguments select
int bn_part_rows(const IgemmArgs& a, bool bf16) {
  if (!bf16) return 128;
  const int64_t xb = (int64_t)a.N * a.H * a.W * a.C * 2, wb = (int64_t)a.K * a.wrow * 2;
  const int bn = big_tile_cols(a, xb, wb);
  return bn >= 128 ? big_tile_rows(bn) : bn == 64 ? 64 : 128;  // one per tile / 64-row wave row / 128-row tile
}

template <typename T, typename OutT>
int launch_igemm(const IgemmArgs& a, hipStream_t st) {
  RN_CHECK_ARG((int64_t)a.N * a.H * a.W * a.C < (1ll << 31), "gathered tensor exceeds 2^31 elements");
  RN_CHECK_ARG((int64_t)a.K * a.wrow < (1ll << 31), "weight matrix exceeds 2^31 elements");
  int maxMc = 0;
  for (int z = 0; z < a.ncls; ++z) maxMc = std::max(maxMc, a.N * a.cls[z].Pc * a.cls[z].Qc);
  if (maxMc == 0) return 0;
  IgemmArgs b = a;
  b.diag_l1 = g_tune[RN_TUNE_DIAG_IGEMM_L1];
  b.sched = g_tune[RN_TUNE_IGEMM_SCHED];
  b.epi_sync = g_tune[RN_TUNE_EPI_SYNC];
  b.nt_store = (g_tune[RN_TUNE_BN_NT] & 16) != 0;
  b.prio = g_tune[RN_TUNE_IGEMM_PRIO];
  const int64_t xb = (int64_t)a.N * a.H * a.W * a.C * (int64_t)sizeof(T);
  const int64_t wb = (int64_t)a.K * a.wrow * (int64_t)sizeof(T);
  b.x_bytes = (int)std::min<int64_t>(xb, INT32_MAX);
  b.w_bytes = (int)std::min<int64_t>(wb, INT32_MAX);
  // LDS-DMA staging (opt-in, rn_set_tuning 1) unless the input transform needs a register pass or an operand is
  // too large for 32-bit buffer offsets
  int max_taps = 0;
  for (int z = 0; z < a.ncls; ++z) max_taps = std::max(max_taps, a.cls[z].nr * a.cls[z].ns);
  const bool dma = g_tune[RN_TUNE_IGEMM_DMA] > 0 && !a.in_sc && !b.diag_l1 && xb < INT32_MAX && wb < INT32_MAX &&
                   max_taps <= 64;
  if constexpr (std::is_same<T, bf16_t>::value && std::is_same<OutT, bf16_t>::value) {
    const int epi = a.stats ? 1 : a.bnred ? (a.bn_clip ? 4 : 2) : a.bn_coef ? 3 : 0;
    const int bn = big_tile_cols(a, xb, wb);
    RN_CHECK_ARG((epi != 3 || bn >= 128) && (epi != 4 || bn >= 64),
                 "this dgrad epilogue needs an LDS-DMA tile");
    const bool m32 = g_tune[RN_TUNE_IGEMM_MFMA] != 1;
    // persistent tiles (rn_set_tuning 10 = workgroups, a multiple of 8): only where the grid is larger
    b.ntiles = 0;
    auto persist = [&](dim3& grid) {
      const int g = g_tune[RN_TUNE_IGEMM_PERSIST] / 8 * 8;
      if (g > 0 && (int)grid.x > g) {
        b.ntiles = (int)grid.x;
        grid.x = (unsigned)g;
      }
    };
    if (bn == 64 && (epi == 0 || !a.smallc)) {
      b.ntn = (int)ceil_div(a.K, 64);
      if (a.bnred) b.mt_max = (int)ceil_div(maxMc, 64);  // BN partials per 64-row wave row
      dim3 grid((unsigned)(ceil_div(maxMc, 256) * b.ntn), 1, a.ncls);
      persist(grid);
      // block-diagonal grouped tile (GD: the MFMAs of off-diagonal k-steps skipped)
      const bool gd = m32 && a.gred > 0 && a.gcol == a.gred && a.gcol <= 32 && a.cblk == 64 &&
                      g_tune[RN_TUNE_IGEMM_GD] != 1;
      if (a.smallc) hipLaunchKernelGGL((igemm_big_kernel<64, 2, 0, true, 256, 1>), grid, dim3(256), 0, st, b);
      else if (epi == 1 && a.in_sc)  // (big_tile_cols: C = 64)
        hipLaunchKernelGGL((igemm_big_kernel<64, 2, 1, true, 256, 0, 0, 2>), grid, dim3(256), 0, st, b);
      else if (epi == 0 && a.in_sc)
        hipLaunchKernelGGL((igemm_big_kernel<64, 2, 0, true, 256, 0, 0, 2>), grid, dim3(256), 0, st, b);
      else if (epi == 1 && gd)
        hipLaunchKernelGGL((igemm_big_kernel<64, 2, 1, true, 256, 0, 0, 0, 0, 1>), grid, dim3(256), 0, st, b);
      else if (epi == 2 && gd)
        hipLaunchKernelGGL((igemm_big_kernel<64, 2, 2, true, 256, 0, 0, 0, 0, 1>), grid, dim3(256), 0, st, b);
      else if (epi == 1) hipLaunchKernelGGL((igemm_big_kernel<64, 2, 1, true>), grid, dim3(256), 0, st, b);
      else if (epi == 2) hipLaunchKernelGGL((igemm_big_kernel<64, 2, 2, true>), grid, dim3(256), 0, st, b);
      else if (epi == 4) hipLaunchKernelGGL((igemm_big_kernel<64, 2, 4, true>), grid, dim3(256), 0, st, b);
      else if (gd)
        hipLaunchKernelGGL((igemm_big_kernel<64, 2, 0, true, 256, 0, 0, 0, 0, 1>), grid, dim3(256), 0, st, b);
      else if (m32) hipLaunchKernelGGL((igemm_big_kernel<64, 2, 0, true>), grid, dim3(256), 0, st, b);
      else hipLaunchKernelGGL((igemm_big_kernel<64, 2, 0, false>), grid, dim3(256), 0, st, b);
      return rn_check_launch("igemm_big64");
    }
    if (bn >= 128) {
      const int bm = big_tile_rows(bn);
      RN_CHECK_ARG(!(a.stats || a.bnred) || bm == bn_part_rows(a, true), "BN partial rows mismatch");
      if (a.bnred) b.mt_max = (int)ceil_div(maxMc, bm);
      b.ntn = (int)ceil_div(a.K, bn);
      dim3 grid((unsigned)(ceil_div(maxMc, bm) * b.ntn), 1, a.ncls);
      persist(grid);
#define RN_BIG(BNV, NB, M, R)                                                                                 \
  if (epi == 0) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 0, M, R>), grid, dim3(512), 0, st, b);        \
  else if (epi == 1) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 1, M, R>), grid, dim3(512), 0, st, b);   \
  else if (epi == 2) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 2, M, R>), grid, dim3(512), 0, st, b);   \
  else if (epi == 3) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 3, M, R>), grid, dim3(512), 0, st, b);   \
  else hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 4, M, R>), grid, dim3(512), 0, st, b);
      if (bn == 128 && bm == 224 && w4_tile(a)) {  // two 4-wave workgroups per CU
        dim3 g4((unsigned)(ceil_div(maxMc, 224) * b.ntn), 1, 1);
        const int pw = g_tune[RN_TUNE_IGEMM_PERSIST] / 8 * 16;
        b.ntiles = 0;
        if (pw > 0 && (int)g4.x > pw) {
          b.ntiles = (int)g4.x;
          g4.x = (unsigned)pw;
        }
        if (a.in_sc) {
          if (epi == 0) hipLaunchKernelGGL((igemm_big_kernel<128, 1, 0, false, 224, 0, 0, 1, 1>), g4, dim3(256), 0, st, b);
          else hipLaunchKernelGGL((igemm_big_kernel<128, 1, 1, false, 224, 0, 0, 1, 1>), g4, dim3(256), 0, st, b);
        } else if (epi == 0) hipLaunchKernelGGL((igemm_big_kernel<128, 1, 0, false, 224, 0, 0, 0, 1>), g4, dim3(256), 0, st, b);
        else if (epi == 1) hipLaunchKernelGGL((igemm_big_kernel<128, 1, 1, false, 224, 0, 0, 0, 1>), g4, dim3(256), 0, st, b);
        else if (epi == 2) hipLaunchKernelGGL((igemm_big_kernel<128, 1, 2, false, 224, 0, 0, 0, 1>), g4, dim3(256), 0, st, b);
        else if (epi == 3) hipLaunchKernelGGL((igemm_big_kernel<128, 1, 3, false, 224, 0, 0, 0, 1>), g4, dim3(256), 0, st, b);
        else hipLaunchKernelGGL((igemm_big_kernel<128, 1, 4, false, 224, 0, 0, 0, 1>), g4, dim3(256), 0, st, b);
        return rn_check_launch("igemm_big_w4");
      }
      if (a.in_sc) {  // (big_tile_cols: 224 rows, forward)
        RN_CHECK_ARG(bm == 224 && epi != 2, "input transform tile");
        if (bn == 256) {
          if (epi == 0) hipLaunchKernelGGL((igemm_big_kernel<256, 2, 0, false, 224, 0, 0, 1>), grid, dim3(512), 0, st, b);
          else hipLaunchKernelGGL((igemm_big_kernel<256, 2, 1, false, 224, 0, 0, 1>), grid, dim3(512), 0, st, b);
        } else {
          if (epi == 0) hipLaunchKernelGGL((igemm_big_kernel<128, 3, 0, false, 224, 0, 0, 1>), grid, dim3(512), 0, st, b);
          else hipLaunchKernelGGL((igemm_big_kernel<128, 3, 1, false, 224, 0, 0, 1>), grid, dim3(512), 0, st, b);
        }
      } else if (bm == 224) {
        if (bn == 256) {
          RN_BIG(256, 2, false, 224)
        } else {
          RN_BIG(128, 3, false, 224)
        }
      } else if (bn == 256 && m32) {
        RN_BIG(256, 2, true, 256)
      } else if (bn == 256) {
        RN_BIG(256, 2, false, 256)
      } else if (m32) {
        RN_BIG(128, 3, true, 256)
      } else {
        RN_BIG(128, 3, false, 256)
      }
#undef RN_BIG
      return rn_check_launch("igemm_big");
    }
  }
  if (std::is_same<T, bf16_t>::value && std::is_same<OutT, float>::value && g_tune[RN_TUNE_DETERMINISTIC] != 1 &&
      a.ncls == 1 && !a.smallc && !a.add &&
      !a.stats && !a.bnred && !a.in_sc && a.gred == 0 && a.cls[0].nr * a.cls[0].ns == 1 && a.K > 64) {
    // split-K for small grids (the FC forward: 256 x 1000 over 2048 = 16 tiles of 32 stages)
    const int64_t tiles = ceil_div(maxMc, 128) * ceil_div(a.K, 128);
    const int nst = (int)ceil_div(a.cblk, 64);
    if (tiles < 128 && nst >= 8) {
      b.ksplit = (int)std::min<int64_t>(nst / 4, std::max<int64_t>(1, 256 / tiles));
      b.ntn = (int)ceil_div(a.K, 128);
      if (hipMemsetAsync(b.y, 0, (size_t)maxMc * a.ldo * sizeof(float), st) != hipSuccess)
        return rn_check_launch("igemm_splitk_zero");
      dim3 grid((unsigned)(ceil_div(maxMc, 128) * b.ntn), (unsigned)b.ksplit, 1);
      hipLaunchKernelGGL((igemm_kernel<T, OutT, 128, 128, false>), grid, dim3(256), 0, st, b);
      return rn_check_launch("igemm_splitk");
    }
  }
  if (a.K <= 64 || a.gred > 0) {  // grouped: the block width is RN_GROUP_BLOCK
    b.ntn = (int)ceil_div(a.K, 64);
    dim3 grid((unsigned)(ceil_div(maxMc, 128) * b.ntn), 1, a.ncls);
    if (dma) hipLaunchKernelGGL((igemm_kernel<T, OutT, 128, 64, true>), grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL((igemm_kernel<T, OutT, 128, 64, false>), grid, dim3(256), 0, st, b);
  } else {
    b.ntn = (int)ceil_div(a.K, 128);
    dim3 grid((unsigned)(ceil_div(maxMc, 128) * b.ntn), 1, a.ncls);
    if (dma) hipLaunchKernelGGL((igemm_kernel<T, OutT, 128, 128, true>), grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL((igemm_kernel<T, OutT, 128, 128, false>), grid, dim3(256), 0, st, b);
  }
  return rn_check_launch("igemm");
}

// int8 forward tile columns: the 4-wave 256x64 tile for <= 64 output channels, else the bf16 family's
// rule (256 columns when the output has >= 256 and the grid keeps >= 192 tiles, else 128)
int i8_tile_cols(const IgemmArgs& a) {
  if (a.K <= 64) return 64;
  const int64_t rows = ceil_div((int64_t)a.N * a.cls[0].Pc * a.cls[0].Qc, 256);
  return (a.K >= 256 && rows * ceil_div(a.K, 256) >= 192) ? 256 : 128;
}

// int8 codes (Q8) on igemm_big_kernel: x / w are int8 with channel strides in bytes
int launch_igemm_i8(const IgemmArgs& a, bool f32out, hipStream_t st) {
  const int64_t xb = (int64_t)a.N * a.H * a.W * a.C, wb = (int64_t)a.K * a.wrow;
  RN_CHECK_ARG(xb < INT32_MAX && wb < INT32_MAX, "int8 operands exceed 32-bit buffer offsets");
  RN_CHECK_ARG(a.C % 16 == 0 && a.gred == 0 && !a.smallc && !a.in_sc && !a.bias && a.ncls == 1,
               "int8 convolution: dense, channel stride a multiple of 16, no bias / input transform");
  RN_CHECK_ARG(a.cls[0].nr * a.cls[0].ns <= 32, "int8 convolution: at most 32 taps");
  const int Mc = a.N * a.cls[0].Pc * a.cls[0].Qc;
  if (Mc == 0) return 0;
  IgemmArgs b = a;
  b.sched = g_tune[RN_TUNE_IGEMM_SCHED];
  b.epi_sync = g_tune[RN_TUNE_EPI_SYNC];
  b.nt_store = (g_tune[RN_TUNE_BN_NT] & 16) != 0;
  b.x_bytes = (int)xb;
  b.w_bytes = (int)wb;
  b.ntiles = 0;
  const int epi = a.stats ? (a.stats_mm ? 5 : 1) : 0;
  const int bn = i8_tile_cols(a);
  const int bm = bn == 64 ? 256 : 224;
  b.ntn = (int)ceil_div(a.K, bn);
  dim3 grid((unsigned)(ceil_div(Mc, bm) * b.ntn), 1, 1);
  const int g = g_tune[RN_TUNE_IGEMM_PERSIST] / 8 * 8;
  if (g > 0 && (int)grid.x > g) {
    b.ntiles = (int)grid.x;
    grid.x = (unsigned)g;
  }
#define RN_I8(BNV, NB, R, T)                                                                                        \
  if (f32out) {                                                                                                    \
    if (epi) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 1, false, R, 0, 2>), grid, dim3(T), 0, st, b);        \
    else hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 0, false, R, 0, 2>), grid, dim3(T), 0, st, b);            \
  } else {                                                                                                         \
    if (epi == 5) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 5, false, R, 0, 1>), grid, dim3(T), 0, st, b);   \
    else if (epi) hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 1, false, R, 0, 1>), grid, dim3(T), 0, st, b);   \
    else hipLaunchKernelGGL((igemm_big_kernel<BNV, NB, 0, false, R, 0, 1>), grid, dim3(T), 0, st, b);            \
  }
  if (bn == 64) {
    RN_I8(64, 2, 256, 256)
  } else if (bn == 128) {
    RN_I8(128, 3, 224, 512)
  } else {
    RN_I8(256, 2, 224, 512)
  }
#undef RN_I8
  return rn_check_launch("igemm_i8");
}

// int8 codes of the KRSC compute copy: round(w / unit) (Quantization_int8 weight path, per tensor:
// symbol/quant_ops.py:17-31, unit = max|w| / qmax), zero in the channel padding
__global__ void pack_krsc_i8_kernel(const float* __restrict__ wm, const float* __restrict__ unit,
                                    int8_t* __restrict__ out, int K, int RS, int creal, int c) {
  const float u = *unit;
  const int64_t total = (int64_t)K * RS * c;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % c);
    const int64_t kt = i / c;
    const float v = ci < creal ? wm[kt * creal + ci] : 0.f;
    out[i] = (int8_t)(u > 0.f ? (int)roundf(v / u) : 0);
  }
}

// Does the grouped convolution d run the direct kernel in mode 0 (forward) / 1 (data gradient)? Its
// compute copy of that mode is then the compact one (pack_group_direct_kernel). Where it pays (measured,
// ResNeXt-50 at batch 256): 4 channels per group -- forward and data gradient, stride 1 / 2 -- and the
// 8-per-group stride-2 layers; with 8 (stride 1) or 16 per group the v_dot2 work outgrows the memory
// time and the block-diagonal MFMA tiles win.
bool gd_direct_shape(const rn_conv_desc* d, int mode) {
  if (!d || d->dtype != RN_BF16 || d->groups <= 1) return false;
  const int cpg = d->c / d->groups;
  if (d->c != d->c_real || d->k != d->c || d->k_pad != d->k || d->c % d->groups || (cpg != 4 && cpg != 8)) return false;
  if (d->r != 3 || d->s != 3 || d->pad_h != 1 || d->pad_w != 1 || d->stride_h != d->stride_w) return false;
  if (d->c % 8 || 64 % (d->c / 8) || (int64_t)(d->c / 8) * (9 * cpg + 1) * 16 > 64 * 1024) return false;
  if (cpg == 8) return (mode == 0 || mode == 1) && d->stride_h == 2;  // (stride 1: the MFMA tile wins)
  return (mode == 0 || mode == 1) && (d->stride_h == 1 || d->stride_h == 2);
}
// The choice is recorded in the descriptor by rn_conv_desc_init (rn_set_tuning 15 = 1 at that time:
// the block-diagonal path), so the packs and the launches of one descriptor always agree on the
// layout of its copies, whatever the tuning key says later.
bool gd_direct_ok(const rn_conv_desc* d, int mode) {
  return d && d->grouped_direct == 1 && gd_direct_shape(d, mode);
}

// ---- 3x3 / stride 1 / pad 1 convolution of 64 channels into 64 over image bands in LDS (ResNet-50
// stage 1's conv2 forward and data gradient, symbol/resnet.py:24-27; rn_set_tuning 26 = 1: off). The implicit
// GEMM DMAs every input element once per tap (nine 64-channel K-tiles from L2); here a persistent
// workgroup keeps all nine taps' weights in LDS (72 KB, [tap][out][in]) and double-buffers bands of
// six input rows (four output rows and their halo, 58 pixel slots per row: the halo columns and rows
// outside the image zero-filled by the DMA; 44 KB each, 160 KB in all), so each input element is loaded
// 1.5 times and every tap reads it from LDS. Seven waves: wave w owns 16-pixel blocks 2w, 2w + 1 of the
// band's 4 W <= 224 pixels, all 64 output channels (per (tap, k-step) 6 fragment reads for 8 MFMAs, the
// next step's reads issued before this step's MFMAs); the MFMA operands are swapped so a lane's
// accumulator holds four consecutive channels of one pixel (one 8-byte store per block). Data gradient
// (FLIP): dy through the CRSK copy with the taps mirrored, dx[p] = sum dy[p + t - 1] w[8 - t]. ResNet-50
// stage 1 (tools/conv_bench.py, same box): forward 113.7 -> 63.7 us, data gradient 123.4 -> 77.9 us.
struct BandArgs {
  const float *in_sc, *in_sh;  // (XF) the producing BatchNorm+ReLU, applied to the landed band
  const void* x;  // [N][H][W][64] bf16
  const void* w;  // [64][9][64] bf16: out, tap, in
  void* y;        // [N][H][W][64] bf16
  int N, H, W, hb, nbands, x_bytes, y_bytes;
};
constexpr int kBandSlots = 58;                     // pixel slots per band row (W + 2 halo columns, W <= 56)
constexpr int kBandRows = 6;                       // 4 output rows + the halo rows
constexpr int kBandChunks = 2816;                  // 16-byte chunks per buffer (6 x 58 x 8 = 2784, rounded
constexpr int kBandBytes = kBandChunks * 16;       // up to whole 64-lane DMA instructions: 44)
template <int FLIP, int XF = 0>
__global__ __launch_bounds__(448, 1) void conv3x3c64_band_kernel(BandArgs p) {
  static_assert(!(FLIP && XF), "the input transform is a forward one");
  __shared__ __attribute__((aligned(16))) uint4 smem[(2 * kBandBytes + 9 * 64 * 128) / 16];  // = 160 KB
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;  // 7 waves: wave w = pixel blocks 2w, 2w + 1
  const v4i rs_x = make_rsrc(p.x, (uint32_t)p.x_bytes);
  const v4i rs_w = make_rsrc(p.w, 64 * 9 * 64 * 2);
  const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.y_bytes, 0x00020000);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  constexpr uint32_t kW = 2 * kBandBytes;  // weights after the two band buffers
  // the weights: 576 rows (tap, out) x 8 chunks, chunk phys of row r holding in-channel chunk phys ^ (r & 7);
  // 72 pieces over waves 0-5
  if (wid < 6) {
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int ins = wid * 12 + j, chunk = ins * 64 + lane;
      const int row = chunk >> 3, tap = row >> 6, o = row & 63;
      const int logical = (chunk & 7) ^ (row & 7);
      dma16_asm(rs_w, lds0 + kW + ins * 1024, (uint32_t)(((o * 9 + (FLIP ? 8 - tap : tap)) * 64 + logical * 8) * 2));
    }
  }
  // band b -> buffer bb (44 pieces over waves 0-3): slot (row br, column bc) holds input row h0 - 1 + br,
  // column bc - 1, its chunk phys holding channel chunk phys ^ (slot & 7)
  auto issue_band = [&](int b, int bb) __attribute__((always_inline)) {
    if (wid >= 4) return;
    const int n = b / p.hb, h0 = (b - n * p.hb) * 4;
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const int ins = wid * 11 + j, chunk = ins * 64 + lane;
      const int pix = chunk >> 3, br = pix / kBandSlots, bc = pix - br * kBandSlots;
      const int h = h0 - 1 + br, wc = bc - 1;
      const int logical = (chunk & 7) ^ (pix & 7);
      const bool ok = br < kBandRows && (unsigned)h < (unsigned)p.H && (unsigned)wc < (unsigned)p.W;
      dma16_asm(rs_x, lds0 + bb * kBandBytes + ins * 1024,
                ok ? (uint32_t)((((n * p.H + h) * p.W + wc) * 64 + logical * 8) * 2) : kOob);
    }
  };
  // this lane's output pixels bk * 16 + (lane & 15) (bk = 2 wid + i) = (orow, ocol); for tap (r, s) the
  // input sits in slot (orow + r) * 58 + ocol + s, at byte ab[i][r][s] (+ 64 for k-step 1); weight block j
  // at wbj[j] + tap * 8192
  const int q = lane >> 4, c = lane & 15;
  int ab[2][3][3], orow[2], ocol[2], pp[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    pp[i] = (2 * wid + i) * 16 + c;
    orow[i] = min(pp[i] / p.W, 3);
    ocol[i] = pp[i] - orow[i] * p.W;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const int slot = min((orow[i] + r) * kBandSlots + min(ocol[i] + sx, kBandSlots - 1), kBandRows * kBandSlots - 1);
        ab[i][r][sx] = slot * 128 + ((q ^ (slot & 7)) << 4);
      }
  }
  int wbj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = j * 16 + c;
    wbj[j] = (int)kW + o * 128 + ((q ^ (o & 7)) << 4);
  }
  const char* lds = reinterpret_cast<const char*>(smem);
  int it = 0;
  int b = blockIdx.x;
  if (b < p.nbands) issue_band(b, 0);
  for (; b < p.nbands; b += gridDim.x, ++it) {
    const int bb = it & 1;
    if (it == 0) wait_vmcnt<0>();
    else wait_vmcnt<8>();  // (the previous band's 8 stores may stay in flight)
    __syncthreads();       // the band has landed for every wave; every wave is done with the other buffer
    const int n = b / p.hb, h0 = (b - n * p.hb) * 4;
    if constexpr (XF) {
      // max(x * sc + sh, 0) rounded to bf16 in place, as bn_apply_kernel stores it; the zero halo (the
      // convolution pads the activation) stays zero
      uint4* band = smem + bb * (kBandBytes / 16);
      for (int i = tid; i < kBandRows * kBandSlots * 8; i += 448) {
        const int pix = i >> 3, br = pix / kBandSlots, bc = pix - br * kBandSlots;
        if ((unsigned)(h0 - 1 + br) >= (unsigned)p.H || (unsigned)(bc - 1) >= (unsigned)p.W) continue;
        const int ch = ((i & 7) ^ (pix & 7)) * 8;
        float f[8];
        chunk_to_f(band[i], f, (const bf16_t*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], p.in_sc[ch + e], p.in_sh[ch + e]), 0.f);
        band[i] = f_to_chunk(f, (const bf16_t*)nullptr);
      }
      __syncthreads();
    }
    if (b + (int)gridDim.x < p.nbands) issue_band(b + gridDim.x, bb ^ 1);
    v4f acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    const int boff = bb * kBandBytes;
    // 18 steps (tap, k-step), each 6 fragment reads (2 pixel blocks, 4 weight blocks) for 8 MFMAs; step i + 1's
    // reads are issued before step i's MFMAs
    uint4 fa[2][2], fb[2][4];
    auto ld = [&](int step, int slot) __attribute__((always_inline)) {
      const int t = step >> 1, ks = step & 1, r = t / 3, sx = t % 3;
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[slot][i] = *reinterpret_cast<const uint4*>(lds + boff + (ab[i][r][sx] ^ (ks * 64)));
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[slot][j] = *reinterpret_cast<const uint4*>(lds + ((wbj[j] + t * 8192) ^ (ks * 64)));
    };
    ld(0, 0);
#pragma unroll
    for (int step = 0; step < 18; ++step) {
      if (step + 1 < 18) ld(step + 1, (step + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);  // (hipcc otherwise sinks every read next to its MFMA)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mfma_slab<bf16_t>(acc[i][j], fb[step & 1][j], fa[step & 1][i]);  // (swapped: lane = pixel, 4 channels)
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int h = h0 + orow[i];
      const bool ok = pp[i] < 4 * p.W && h < p.H;
      const int obase = (((n * p.H + h) * p.W + ocol[i]) * 64 + 4 * q) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        const uint32_t voff = ok ? (uint32_t)(obase + j * 32) : 0x80000000u;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo, hi}, rs_y, voff, 0, 0);
      }
    }
  }
}

// The int8 forward of the same layer (symbol/resnet_int8.py: the quantized stage-1 conv2): x and the
// weights as int8 codes (64-byte pixel slots, one 16x16x64 i8 MFMA k-step per tap), y = unit_x * unit_w *
// the exact int32 sums (igemm_big_kernel Q8's epilogue, so bit-identical to it). 80 KB of LDS: two
// workgroups per CU. 64-byte slots: chunk phys of slot s holds channel chunk phys ^ ((s >> 1) & 3).
constexpr int kBand8Chunks = 1408;  // 6 x 58 x 4 = 1392, rounded up to 22 whole 64-lane DMA instructions
constexpr int kBand8Bytes = kBand8Chunks * 16;
struct Band8Args {
  const void* x;  // [N][H][W][64] int8 codes
  const void* w;  // [64][9][64] int8 codes
  void* y;        // [N][H][W][64] bf16
  const float *ux, *uw;
  int N, H, W, hb, nbands, x_bytes, y_bytes;
};
__global__ __launch_bounds__(448, 2) void conv3x3c64_band_i8_kernel(Band8Args p) {
  __shared__ __attribute__((aligned(16))) uint4 smem[(2 * kBand8Bytes + 9 * 64 * 64) / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const v4i rs_x = make_rsrc(p.x, (uint32_t)p.x_bytes);
  const v4i rs_w = make_rsrc(p.w, 64 * 9 * 64);
  const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.y_bytes, 0x00020000);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  constexpr uint32_t kW = 2 * kBand8Bytes;
  if (wid < 6) {  // 576 rows (tap, out) x 4 chunks = 36 pieces over waves 0-5
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int ins = wid * 6 + j, chunk = ins * 64 + lane;
      const int row = chunk >> 2, tap = row >> 6, o = row & 63;
      const int logical = (chunk & 3) ^ ((row >> 1) & 3);
      dma16_asm(rs_w, lds0 + kW + ins * 1024, (uint32_t)((o * 9 + tap) * 64 + logical * 16));
    }
  }
  auto issue_band = [&](int b, int bb) __attribute__((always_inline)) {
    if (wid >= 2) return;  // 22 pieces over waves 0-1
    const int n = b / p.hb, h0 = (b - n * p.hb) * 4;
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const int ins = wid * 11 + j, chunk = ins * 64 + lane;
      const int pix = chunk >> 2, br = pix / kBandSlots, bc = pix - br * kBandSlots;
      const int h = h0 - 1 + br, wc = bc - 1;
      const int logical = (chunk & 3) ^ ((pix >> 1) & 3);
      const bool ok = br < kBandRows && (unsigned)h < (unsigned)p.H && (unsigned)wc < (unsigned)p.W;
      dma16_asm(rs_x, lds0 + bb * kBand8Bytes + ins * 1024,
                ok ? (uint32_t)(((n * p.H + h) * p.W + wc) * 64 + logical * 16) : kOob);
    }
  };
  const int q = lane >> 4, c = lane & 15;
  int ab[2][9], orow[2], ocol[2], pp[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    pp[i] = (2 * wid + i) * 16 + c;
    orow[i] = min(pp[i] / p.W, 3);
    ocol[i] = pp[i] - orow[i] * p.W;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int slot = min((orow[i] + t / 3) * kBandSlots + min(ocol[i] + t % 3, kBandSlots - 1), kBandRows * kBandSlots - 1);
      ab[i][t] = slot * 64 + ((q ^ ((slot >> 1) & 3)) << 4);
    }
  }
  int wbj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = j * 16 + c;
    wbj[j] = (int)kW + o * 64 + ((q ^ ((o >> 1) & 3)) << 4);  // + tap * 4096
  }
  const float qs = *p.ux * *p.uw;
  const char* lds = reinterpret_cast<const char*>(smem);
  int it = 0;
  int b = blockIdx.x;
  if (b < p.nbands) issue_band(b, 0);
  for (; b < p.nbands; b += gridDim.x, ++it) {
    const int bb = it & 1;
    if (it == 0) wait_vmcnt<0>();
    else wait_vmcnt<8>();
    __syncthreads();
    if (b + (int)gridDim.x < p.nbands) issue_band(b + gridDim.x, bb ^ 1);
    v4i acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
    const int boff = bb * kBand8Bytes;
    uint4 fa[2][2], fb[2][4];
    auto ld = [&](int t, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[slot][i] = *reinterpret_cast<const uint4*>(lds + boff + ab[i][t]);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[slot][j] = *reinterpret_cast<const uint4*>(lds + wbj[j] + t * 4096);
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4 a8 = fb[t & 1][j], b8 = fa[t & 1][i];
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(*reinterpret_cast<const v4i*>(&a8),
                                                             *reinterpret_cast<const v4i*>(&b8), acc[i][j], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    const int n = b / p.hb, h0 = (b - n * p.hb) * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int h = h0 + orow[i];
      const bool ok = pp[i] < 4 * p.W && h < p.H;
      const int obase = (((n * p.H + h) * p.W + ocol[i]) * 64 + 4 * q) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = (uint32_t)f2bf((float)acc[i][j][0] * qs) | ((uint32_t)f2bf((float)acc[i][j][1] * qs) << 16);
        const uint32_t hi = (uint32_t)f2bf((float)acc[i][j][2] * qs) | ((uint32_t)f2bf((float)acc[i][j][3] * qs) << 16);
        const uint32_t voff = ok ? (uint32_t)(obase + j * 32) : 0x80000000u;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo, hi}, rs_y, voff, 0, 0);
      }
    }
  }
}

// geometry of a direct grouped launch (mode 0 forward, 1 data gradient): fills a's shape fields,
// returns the workgroups (also the BatchNorm-reduction partials of a RED data gradient)
int gd_geometry(const rn_conv_desc* d, int mode, GdArgs& a) {
  a.C = d->c;
  if (mode == 0) { a.H = d->h; a.W = d->w; a.P = d->p; a.Q = d->q; a.pad = d->pad_h; }
  else { a.H = d->p; a.W = d->q; a.P = d->h; a.Q = d->w; a.pad = d->r - 1 - d->pad_h; }
  int lcpr = 0;
  while ((8 << lcpr) < d->c) ++lcpr;
  a.lcpr = lcpr;
  const int cpg = d->c / d->groups;
  const int stride = mode == 0 ? d->stride_h : 1;
  const bool s2t = mode == 1 && d->stride_h == 2;  // the transposed stride-2 data gradient
  const int PL = s2t ? 8 : cpg == 4 && stride == 1 ? 8 : 4;
  a.qb = (a.Q + PL - 1) / PL;
  const int64_t items = (int64_t)d->n * a.P * a.qb;
  a.items = (uint32_t)std::min<int64_t>(items, UINT32_MAX);
  const int plw = 64 >> lcpr;
  const int64_t want = (items + 4 * plw - 1) / (4 * plw);
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, 1024));
}

int gd_launch(const rn_conv_desc* d, int mode, const void* x, const void* w, void* y, const void* add,
              hipStream_t st, const GdArgs* red = nullptr) {
  GdArgs a{};
  if (red) a = *red;  // (data gradient: the BatchNorm reduction fields)
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.y = (bf16_t*)y; a.add = (const bf16_t*)add;
  const int blocks = gd_geometry(d, mode, a);
  RN_CHECK_ARG((int64_t)d->n * a.P * a.qb < INT32_MAX && (int64_t)d->n * a.H * a.W * a.C < INT32_MAX,
               "grouped direct: tensor too large");
  a.fdQB = make_fastdiv(a.qb); a.fdP = make_fastdiv(a.P);
  const int cpg = d->c / d->groups;
  const int stride = mode == 0 ? d->stride_h : 1;
  const bool s2t = mode == 1 && d->stride_h == 2;
  const size_t lds = (size_t)(d->c / 8) * (9 * cpg + 1) * 16;  // (kGdWStride: one pad row per chunk)
  const bool rd = a.bnred != nullptr;
  RN_CHECK_ARG(!rd || (mode == 1 && d->c <= kGdRedMaxC), "grouped direct BN reduction: data gradient only");
  if (s2t) {
    if (cpg == 4 && rd) hipLaunchKernelGGL((grouped_dgrad_s2_kernel<4, 8, true>), dim3(blocks), dim3(256), lds, st, a);
    else if (cpg == 4) hipLaunchKernelGGL((grouped_dgrad_s2_kernel<4, 8>), dim3(blocks), dim3(256), lds, st, a);
    else if (rd) hipLaunchKernelGGL((grouped_dgrad_s2_kernel<8, 8, true>), dim3(blocks), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((grouped_dgrad_s2_kernel<8, 8>), dim3(blocks), dim3(256), lds, st, a);
  } else if (cpg == 4 && stride == 1) {
    if (rd) hipLaunchKernelGGL((grouped_direct_kernel<4, 1, 8, true>), dim3(blocks), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((grouped_direct_kernel<4, 1, 8>), dim3(blocks), dim3(256), lds, st, a);
  } else if (cpg == 4)
    hipLaunchKernelGGL((grouped_direct_kernel<4, 2, 4>), dim3(blocks), dim3(256), lds, st, a);
  else
    hipLaunchKernelGGL((grouped_direct_kernel<8, 2, 4>), dim3(blocks), dim3(256), lds, st, a);
  return rn_check_launch(mode == 0 ? "grouped_direct_fwd" : "grouped_direct_dgrad");
}

// conv3x3c64_band_kernel for these arguments? (rn_set_tuning 26 = 1: never -- the implicit-GEMM tile)
bool band_ok(const rn_conv_desc* d) {
  return g_tune[RN_TUNE_CONV_BAND] != 1 && d->dtype == RN_BF16 && d->groups <= 1 && d->r == 3 && d->s == 3 &&
         d->stride_h == 1 && d->stride_w == 1 && d->pad_h == 1 && d->pad_w == 1 && d->c == 64 && d->c_real == 64 &&
         d->k == 64 && d->k_pad == 64 && d->w <= 56 && (int64_t)d->n * d->h * d->w * 64 * 2 < INT32_MAX;
}
int band_launch(const rn_conv_desc* d, const void* x, const void* w, void* y, int flip, hipStream_t st,
                const float* in_sc = nullptr, const float* in_sh = nullptr) {
  BandArgs a{};
  a.x = x; a.w = w; a.y = y; a.in_sc = in_sc; a.in_sh = in_sh;
  a.N = d->n; a.H = d->h; a.W = d->w; a.hb = (d->h + 3) / 4; a.nbands = d->n * a.hb;
  a.x_bytes = a.y_bytes = d->n * d->h * d->w * 64 * 2;
  const dim3 grid((unsigned)std::min(a.nbands, chip_cus()));
  if (flip) hipLaunchKernelGGL(conv3x3c64_band_kernel<1>, grid, dim3(448), 0, st, a);
  else if (in_sc) hipLaunchKernelGGL((conv3x3c64_band_kernel<0, 1>), grid, dim3(448), 0, st, a);
  else hipLaunchKernelGGL(conv3x3c64_band_kernel<0>, grid, dim3(448), 0, st, a);
  return rn_check_launch("conv3x3c64_band");
}

// ---- The data gradients of the pre-activation units' conv1 (symbol/resnet.py:17-20: a 1x1 / stride-1
// convolution whose input has 2-4x its output's channels, so its data gradient reduces over K <= 128 channels
// into C >= 256): streaming, not tiled. dx[m][c] = sum_k dy[m][k] w[c][k] (the CRSK copy) is memory-bound
// (2 K MACs per 2 + 2 K / C bytes of dx), and on the 224-row tiles it ran in their epilogue bursts (the BN
// input the reduction reads came in at ~3.5 TB/s). Here a 256-thread workgroup owns 224 rows (one BN-partial
// block, the tiles' granularity) x 128 channels; wave w owns channels 32 w .. + 31 for all 224 rows, in steps of
// 16 rows: v_mfma_f32_16x16x32_bf16 with the weights as the A operand (their fragments in registers for the
// whole kernel) and dy as B, loaded straight from global memory (lane (g, i): 16 bytes of row i). The two MFMA
// blocks interleave their rows' channels (block b, row r -> channel 8 (r >> 2) + 4 b + (r & 3)), so output lane
// (g, i) holds channels 8 g .. 8 g + 7 of row i: every epilogue access is one 16-byte chunk per lane. The next
// step's loads are issued before this step's MFMAs; the workgroups of one row block sit on one XCD (their dy
// rows read into one L2). EPI 0: dx (+ add); 2: + the BatchNorm-backward reduction of the stored dx (as
// igemm_big_kernel EPI 2: sum dz, sum dz (x - mean), dz = dx [x sc + sh > 0]); 3: dx = the BatchNorm backward
// applied to the rounded gradient (EPI 3's formula) + add.
struct D1Args {
  const bf16_t* dy;  // [M][K]
  const bf16_t* w;   // [C][K] (the CRSK copy of a 1x1 conv)
  bf16_t* dx;        // [M][C], nullable with EPI 2 (reduction only)
  const bf16_t* add; // nullable
  const bf16_t* bn_x;
  const float *bn_mean, *coef, *bn_sc, *bn_sh;
  float* part;       // (EPI 2) [M / 224][C][2]
  int M, C, K, relu, ncg;
};
// ADD: p.add is set (a compile-time branch: with a runtime one, hipcc (ROCm 7.2) let the epilogue's first VALU
// read an MFMA result across the branch without the wait states it needs -- stale values in 1 of 8 channels,
// run to run). NH: 32-channel halves per wave (NH = 2: a lane's two 16-byte chunks of a row are 64 bytes apart,
// so each row's 128-byte lines are written whole by one wave).
template <int KS, int EPI, int ADD, int NH>
__global__ __launch_bounds__(256, 2) void dgrad1x1_stream_kernel(D1Args p) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int rb = lid / p.ncg, cg = lid - rb * p.ncg;
  const int m0 = rb * 224, rows = min(224, p.M - m0);
  const int cw = (cg * 4 + wid) * 32 * NH;  // this wave's 32 NH channels
  int c8[NH];                                // this lane's 8-channel chunks
#pragma unroll
  for (int h = 0; h < NH; ++h) c8[h] = cw + 32 * h + 8 * g;
  v8s wf[NH][2][KS];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ch = cw + 32 * h + 8 * (i >> 2) + 4 * b + (i & 3);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        wf[h][b][ks] = *reinterpret_cast<const v8s*>(p.w + (int64_t)ch * p.K + ks * 32 + 8 * g);
    }
  // per-channel constants of the lane's channels (EPI 2: mean, scale, shift; EPI 3: + A, mean dz, A2)
  float mu[NH][8], sc[NH][8], sh[NH][8], ca[NH][8], cm[NH][8], c2[NH][8], s1[NH][8], s2[NH][8];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c8[h] + e;
      s1[h][e] = s2[h][e] = 0.f;
      mu[h][e] = sc[h][e] = sh[h][e] = ca[h][e] = cm[h][e] = c2[h][e] = 0.f;
      if constexpr (EPI == 2) mu[h][e] = p.bn_mean[c];
      if constexpr (EPI >= 2) {
        sc[h][e] = p.bn_sc[c];
        sh[h][e] = p.bn_sh[c];
      }
      if constexpr (EPI == 3) {
        const float4 cf = reinterpret_cast<const float4*>(p.coef)[c];
        ca[h][e] = cf.x; cm[h][e] = cf.y; c2[h][e] = cf.z; mu[h][e] = cf.w;
      }
    }
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  // buffer loads (a row past the block reads zeros through an offset past the buffer): no pointer selects,
  // which hipcc turns into flat loads whose waits (vmcnt(0) with lgkmcnt) would also drain this step's stores
  const __amdgpu_buffer_rsrc_t rs_dy = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, p.M * p.K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)p.bn_x, (short)0, p.M * p.C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_a = __builtin_amdgcn_make_buffer_rsrc((void*)p.add, (short)0, p.M * p.C * 2, 0x00020000);
  // dx through a buffer descriptor too: rows past the block store to an offset past it (dropped), and the
  // reduction-only form (dx = NULL) gets an empty one -- so the step body has no branch
  const __amdgpu_buffer_rsrc_t rs_dx =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dx, (short)0, p.dx ? p.M * p.C * 2 : 0, 0x00020000);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto ld = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off) __attribute__((always_inline)) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
  };
  auto load = [&](int st, uint4 (&d)[KS], uint4 (&xv)[NH], uint4 (&av)[NH]) __attribute__((always_inline)) {
    const int r = st * 16 + i;
    const bool ok = r < rows;
    const uint32_t m = (uint32_t)(m0 + r);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) d[ks] = ld(rs_dy, ok ? (m * p.K + ks * 32 + 8 * g) * 2u : kOob);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      if constexpr (EPI >= 2) xv[h] = ld(rs_x, ok ? (m * p.C + c8[h]) * 2u : kOob);
      if constexpr (ADD) av[h] = ld(rs_a, ok ? (m * p.C + c8[h]) * 2u : kOob);
    }
  };
  const bool norelu = __builtin_amdgcn_readfirstlane(p.relu) == 0;
  uint4 d0[KS], x0[NH], a0[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) x0[h] = a0[h] = z4;
  load(0, d0, x0, a0);
  // fully unrolled, branch-free (14 steps of 16 rows; a short last block's extra rows load zeros and store
  // nothing): hipcc's wait counts then stay exact -- across a loop back-edge or a branch join they became
  // vmcnt(0), draining the previous step's stores and the prefetched loads every step
#pragma unroll
  for (int st = 0; st < 14; ++st) {
    uint4 d1[KS], x1[NH], a1[NH];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) d1[ks] = z4;
#pragma unroll
    for (int h = 0; h < NH; ++h) x1[h] = a1[h] = z4;
    if (st + 1 < 14) load(st + 1, d1, x1, a1);  // (compile-time)
    v4f acc[NH][2];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[h][b] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[h][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[h][b][ks], __builtin_bit_cast(v8s, d0[ks]), acc[h][b],
                                                              0, 0, 0);
    // the MFMA results' read wait states, explicitly (16 >= the 8-pass MFMA's VALU-read hazard), once per step
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7");
    __builtin_amdgcn_sched_barrier(0);
    const int r = st * 16 + i;
    const bool ok = r < rows;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float v[8], xf[8], af[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[h][0][e];
        v[4 + e] = acc[h][1][e];
      }
      chunk_to_f(x0[h], xf, (const bf16_t*)nullptr);
      chunk_to_f(a0[h], af, (const bf16_t*)nullptr);
      uint4 out;
      if constexpr (EPI == 3) {
        float gv[8];
        chunk_to_f(f_to_chunk(v, (const bf16_t*)nullptr), gv, (const bf16_t*)nullptr);  // the gradient as stored
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = norelu ? gv[e] : gv[e] * (fmaf(xf[e], sc[h][e], sh[h][e]) > 0.f ? 1.f : 0.f);
          // spelled out as bn_bwd_apply_kernel is compiled (fma(A, dz - mean dz, -(A2 (x - mean)))): bit-identical
          const float q = c2[h][e] * (xf[e] - mu[h][e]);
          float w = fmaf(ca[h][e], dz - cm[h][e], -q);
          if (ADD) w += af[e];
          v[e] = w;
        }
        out = f_to_chunk(v, (const bf16_t*)nullptr);
      } else {
        if (ADD)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += af[e];
        out = f_to_chunk(v, (const bf16_t*)nullptr);
        if constexpr (EPI == 2) {
          float gv[8];
          chunk_to_f(out, gv, (const bf16_t*)nullptr);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const bool keep = ok & (norelu | (fmaf(xf[e], sc[h][e], sh[h][e]) > 0.f));  // (no short circuit: selects)
            const float dz = keep ? gv[e] : 0.f;
            s1[h][e] += dz;
            s2[h][e] = fmaf(dz, xf[e] - mu[h][e], s2[h][e]);
          }
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{out.x, out.y, out.z, out.w}, rs_dx,
                                             ok ? ((uint32_t)(m0 + r) * p.C + c8[h]) * 2u : kOob, 0, 0);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) d0[ks] = d1[ks];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      x0[h] = x1[h];
      a0[h] = a1[h];
    }
  }
  if constexpr (EPI == 2) {  // the 16 rows lanes of each channel group: xor 1, 2, 4, 8; lane i = 0 stores
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[h][e] += __shfl_xor(s1[h][e], o, 64);
          s2[h][e] += __shfl_xor(s2[h][e], o, 64);
        }
    if (i == 0)
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int64_t o = ((int64_t)rb * p.C + c8[h] + e) * 2;
          p.part[o] = s1[h][e];
          p.part[o + 1] = s2[h][e];
        }
  }
}

// dgrad1x1_stream_kernel for this data gradient? (rn_set_tuning 27 = 1: never -- the 224-row tiles)
bool d1_stream_ok(const rn_conv_desc* d, const float* clip) {
  // (224-row BN partial blocks, as the tiles' with rn_set_tuning 9 = 0)
  return g_tune[RN_TUNE_DGRAD_STREAM] != 1 && g_tune[RN_TUNE_IGEMM_ROWS] != 1 && !clip && d->dtype == RN_BF16 &&
         d->groups <= 1 && d->r == 1 &&
         d->s == 1 && d->stride_h == 1 && d->stride_w == 1 && d->pad_h == 0 && d->pad_w == 0 &&
         d->c == d->c_real && d->c % 128 == 0 && d->k == d->k_pad && (d->k == 64 || d->k == 128) &&
         (int64_t)d->n * d->h * d->w * d->c < INT32_MAX;
}
int d1_stream_launch(const rn_conv_desc* d, int epi, const void* dy, const void* w, void* dx, const void* add,
                     const void* bn_x, const float* mean, const float* coef, const float* sc, const float* sh,
                     int relu, float* part, hipStream_t st) {
  D1Args a{};
  a.dy = (const bf16_t*)dy; a.w = (const bf16_t*)w; a.dx = (bf16_t*)dx; a.add = (const bf16_t*)add;
  a.bn_x = (const bf16_t*)bn_x; a.bn_mean = mean; a.coef = coef; a.bn_sc = sc; a.bn_sh = sh; a.part = part;
  // 64 channels per wave where C % 256 == 0 (rn_set_tuning 27 = 2: 32), except the apply form (EPI 3), whose
  // per-channel coefficients need the registers
  const int nh = (epi != 3 && d->c % 256 == 0 && g_tune[RN_TUNE_DGRAD_STREAM] != 2) ? 2 : 1;
  a.M = d->n * d->h * d->w; a.C = d->c; a.K = d->k; a.relu = relu; a.ncg = d->c / (128 * nh);
  const dim3 grid((unsigned)(ceil_div(a.M, 224) * a.ncg));
#define RN_D1N(KSV, AV, NHV)                                                                                  \
  if (epi == 0) hipLaunchKernelGGL((dgrad1x1_stream_kernel<KSV, 0, AV, NHV>), grid, dim3(256), 0, st, a);    \
  else if (epi == 2) hipLaunchKernelGGL((dgrad1x1_stream_kernel<KSV, 2, AV, NHV>), grid, dim3(256), 0, st, a); \
  else hipLaunchKernelGGL((dgrad1x1_stream_kernel<KSV, 3, AV, 1>), grid, dim3(256), 0, st, a);
#define RN_D1(KSV, AV)     \
  if (nh == 2) {           \
    RN_D1N(KSV, AV, 2)     \
  } else {                 \
    RN_D1N(KSV, AV, 1)     \
  }
  if (d->k == 64) {
    if (add) {
      RN_D1(2, 1)
    } else {
      RN_D1(2, 0)
    }
  } else if (add) {
    RN_D1(4, 1)
  } else {
    RN_D1(4, 0)
  }
#undef RN_D1
#undef RN_D1N
  return rn_check_launch("dgrad1x1_stream");
}

}  // namespace

extern "C" {

int rn_conv_desc_init(rn_conv_desc* d) {
  RN_CHECK_ARG(d != nullptr, "null desc");
  RN_CHECK_ARG(d->dtype == RN_BF16 || d->dtype == RN_F32, "bad dtype");
  RN_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->k > 0, "bad shape");
  RN_CHECK_ARG(d->r > 0 && d->s > 0 && d->stride_h > 0 && d->stride_w > 0, "bad kernel/stride");
  RN_CHECK_ARG(d->pad_h >= 0 && d->pad_w >= 0, "bad pad");
  if (d->groups <= 0) d->groups = 1;
  if (d->c_real <= 0) d->c_real = d->c;
  if (d->k_pad <= 0) d->k_pad = (d->k + 7) / 8 * 8;
  if (d->groups > 1) {
    const int g = d->groups;
    RN_CHECK_ARG(d->c == d->c_real && d->k == d->k_pad, "grouped conv needs unpadded channels");
    RN_CHECK_ARG(d->c % g == 0 && d->k % g == 0, "channels not divisible by num_group");
    const int cpg = d->c / g, kpg = d->k / g;
    auto fits = [](int v) { return RN_GROUP_BLOCK % v == 0 || v % RN_GROUP_BLOCK == 0; };
    RN_CHECK_ARG(fits(cpg) && fits(kpg), "channels per group must divide or be a multiple of 64");
    RN_CHECK_ARG(group_blk(kpg, cpg) % 8 == 0 && group_blk(cpg, kpg) % 8 == 0,
                 "grouped block reduction must be a multiple of 8 channels");
  }
  RN_CHECK_ARG(d->c % 8 == 0, "channel stride must be a multiple of 8");
  RN_CHECK_ARG(d->k_pad % 8 == 0 && d->k_pad >= d->k, "k_pad must be a multiple of 8 >= k");
  RN_CHECK_ARG(d->c_real <= d->c, "c_real > c");
  RN_CHECK_ARG(d->stride_h <= 2 && d->stride_w <= 2, "stride > 2 not supported");
  d->p = (d->h + 2 * d->pad_h - d->r) / d->stride_h + 1;
  d->q = (d->w + 2 * d->pad_w - d->s) / d->stride_w + 1;
  RN_CHECK_ARG(d->p > 0 && d->q > 0, "empty output");
  d->grouped_direct = (g_tune[RN_TUNE_GROUP_DIRECT] != 1 && gd_direct_shape(d, 0)) ? 1 : 0;
  RN_CHECK_ARG((int64_t)d->n * d->h * d->w < (1ll << 31) && (int64_t)d->n * d->p * d->q < (1ll << 31),
               "too many pixels");
  return 0;
}

int64_t rn_conv_weight_numel(const rn_conv_desc* d) {
  return (int64_t)d->k * d->r * d->s * (d->c_real / (d->groups > 0 ? d->groups : 1));
}

int64_t rn_conv_pack_numel(const rn_conv_desc* d, int32_t which) {
  const int64_t RS = (int64_t)d->r * d->s;
  if (gd_direct_ok(d, which)) return (int64_t)d->c * 9 * (d->c / d->groups);  // (compact, see rn.h)
  if (d->groups > 1) {
    const int cpg = d->c / d->groups, kpg = d->k / d->groups;
    return which == 0 ? d->k * RS * group_blk(kpg, cpg) : d->c * RS * group_blk(cpg, kpg);
  }
  return which == 0 ? d->k * RS * d->c : d->c * RS * d->k_pad;
}

int rn_conv_fwd_x(const rn_conv_desc* d, const void* x, const void* w, void* y, int32_t y_dtype,
                  const void* add_src, const float* bias, const float* in_scale, const float* in_shift,
                  float* part, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && w && y, "null argument");
  RN_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "in_scale / in_shift must both be set");
  RN_CHECK_ARG(!in_scale || d->groups == 1, "input transform on a grouped conv");
  if (gd_direct_ok(d, 0)) {
    RN_CHECK_ARG(!bias && !part && y_dtype == RN_BF16, "grouped direct forward: no bias / statistics, bf16 output");
    return gd_launch(d, 0, x, w, y, add_src, as_stream(stream));
  }
  if (band_ok(d) && !add_src && !bias && !part && y_dtype == RN_BF16)
    return band_launch(d, x, w, y, 0, as_stream(stream), in_scale, in_shift);
  IgemmArgs a = make_igemm_args(d, 0);
  a.x = x; a.w = w; a.y = y; a.add = add_src; a.bias = bias; a.stats = part;
  a.in_sc = in_scale; a.in_sh = in_shift;
  RN_CHECK_ARG(!part || d->k % 8 == 0, "BatchNorm statistics need whole 8-channel chunks");
  hipStream_t st = as_stream(stream);
  if (d->dtype == RN_BF16) {
    if (y_dtype == RN_BF16) return launch_igemm<bf16_t, bf16_t>(a, st);
    return launch_igemm<bf16_t, float>(a, st);
  }
  RN_CHECK_ARG(y_dtype == RN_F32, "f32 compute requires f32 output");
  return launch_igemm<float, float>(a, st);
}

int rn_conv_fwd_i8(const rn_conv_desc* d, const void* x_codes, const void* w_codes, void* y, int32_t y_dtype,
                   const void* add_src, const float* x_unit, const float* w_unit, float* part,
                   rn_stream_t stream) {
  return rn_conv_fwd_i8_mm(d, x_codes, w_codes, y, y_dtype, add_src, x_unit, w_unit, part, nullptr, nullptr, stream);
}

int rn_conv_fwd_i8_mm(const rn_conv_desc* d, const void* x_codes, const void* w_codes, void* y, int32_t y_dtype,
                      const void* add_src, const float* x_unit, const float* w_unit, float* part, float* part_mm,
                      const float* mm_sign, rn_stream_t stream) {
  RN_CHECK_ARG(d && x_codes && w_codes && y && x_unit && w_unit, "null argument");
  RN_CHECK_ARG(!part_mm || (part && y_dtype == RN_BF16), "part_mm comes with the BatchNorm partials (bf16 output)");
  RN_CHECK_ARG(!mm_sign || (((uintptr_t)mm_sign & 15) == 0 && d->k % 8 == 0), "mm_sign: 16-byte aligned, k % 8 == 0");
  RN_CHECK_ARG(d->groups <= 1, "int8 convolution is dense");
  RN_CHECK_ARG(y_dtype == RN_BF16 || y_dtype == RN_F32, "bad output dtype");
  RN_CHECK_ARG(!part || d->k % 8 == 0, "BatchNorm statistics need whole 8-channel chunks");
  if (band_ok(d) && !add_src && !part && !part_mm && y_dtype == RN_BF16) {  // (image bands, int8 codes)
    Band8Args b{};
    b.x = x_codes; b.w = w_codes; b.y = y; b.ux = x_unit; b.uw = w_unit;
    b.N = d->n; b.H = d->h; b.W = d->w; b.hb = (d->h + 3) / 4; b.nbands = d->n * b.hb;
    b.x_bytes = d->n * d->h * d->w * 64;
    b.y_bytes = d->n * d->h * d->w * 64 * 2;
    const dim3 grid((unsigned)std::min(b.nbands, 2 * chip_cus()));
    hipLaunchKernelGGL(conv3x3c64_band_i8_kernel, grid, dim3(448), 0, as_stream(stream), b);
    return rn_check_launch("conv3x3c64_band_i8");
  }
  IgemmArgs a = make_igemm_args(d, 0);
  a.smallc = 0;
  a.x = x_codes; a.w = w_codes; a.y = y; a.add = add_src; a.bias = nullptr; a.stats = part; a.stats_mm = part_mm;
  a.mm_sign = mm_sign;
  a.qunit_x = x_unit; a.qunit_w = w_unit;
  return launch_igemm_i8(a, y_dtype == RN_F32, as_stream(stream));
}

int rn_conv_weight_pack_i8(const rn_conv_desc* d, const float* w_master, const float* unit, void* w_codes,
                           rn_stream_t stream) {
  RN_CHECK_ARG(d && w_master && unit && w_codes, "null argument");
  RN_CHECK_ARG(d->groups <= 1, "int8 convolution is dense");
  const int64_t total = (int64_t)d->k * d->r * d->s * d->c;
  hipLaunchKernelGGL(pack_krsc_i8_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), w_master, unit,
                     (int8_t*)w_codes, d->k, d->r * d->s, d->c_real, d->c);
  return rn_check_launch("weight_pack_i8");
}

int rn_conv_fwd(const rn_conv_desc* d, const void* x, const void* w, void* y, int32_t y_dtype,
                const void* add_src, const float* bias, rn_stream_t stream) {
  return rn_conv_fwd_x(d, x, w, y, y_dtype, add_src, bias, nullptr, nullptr, nullptr, stream);
}

int rn_conv_fwd_bnstats(const rn_conv_desc* d, const void* x, const void* w, void* y, int32_t y_dtype,
                        const void* add_src, const float* bias, float* part, rn_stream_t stream) {
  return rn_conv_fwd_x(d, x, w, y, y_dtype, add_src, bias, nullptr, nullptr, part, stream);
}

int32_t rn_conv_tile(const rn_conv_desc* d, int32_t mode) {
  if (d && mode == 2 && d->groups <= 1) return i8_tile_cols(make_igemm_args(d, 0));  // int8 forward
  if (!d || d->dtype != RN_BF16 || (mode != 0 && mode != 1) || gd_direct_ok(d, mode)) return 0;
  const IgemmArgs a = make_igemm_args(d, mode);
  const int64_t xb = (int64_t)a.N * a.H * a.W * a.C * 2, wb = (int64_t)a.K * a.wrow * 2;
  return big_tile_cols(a, xb, wb);
}

int32_t rn_conv_bn_part_rows(const rn_conv_desc* d, int32_t mode) {
  if (d && mode == 2) return rn_conv_tile(d, 2) == 64 ? 64 : 224;  // int8 forward: per wave row / tile
  if (!d || (mode != 0 && mode != 1)) return 0;
  return bn_part_rows(make_igemm_args(d, mode), d->dtype == RN_BF16);
}

int64_t rn_conv_bnstats_blocks(const rn_conv_desc* d) {
  return ceil_div((int64_t)d->n * d->p * d->q, rn_conv_bn_part_rows(d, 0));
}

int64_t rn_conv_bnred_blocks(const rn_conv_desc* d) {
  if (gd_direct_ok(d, 1)) {  // one partial per workgroup of the direct kernel
    GdArgs g{};
    return gd_geometry(d, 1, g);
  }
  IgemmArgs a = make_igemm_args(d, 1);
  int maxMc = 0;
  for (int z = 0; z < a.ncls; ++z) maxMc = std::max(maxMc, a.N * a.cls[z].Pc * a.cls[z].Qc);
  return (int64_t)a.ncls * ceil_div(maxMc, bn_part_rows(a, d->dtype == RN_BF16));
}

int rn_conv_bwd_data_bnred(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx, const void* add_src,
                           const void* bn_x, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                           int32_t relu, float* part, rn_stream_t stream) {
  return rn_conv_bwd_data_bnred_clip(d, dy, w_crsk, dx, add_src, bn_x, bn_mean, bn_scale, bn_shift, relu, nullptr,
                                     part, stream);
}

int rn_conv_bwd_data_bnred_clip(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                                const void* add_src, const void* bn_x, const float* bn_mean, const float* bn_scale,
                                const float* bn_shift, int32_t relu, const float* clip, float* part,
                                rn_stream_t stream) {
  RN_CHECK_ARG(!clip || (part && relu && d && d->dtype == RN_BF16 && rn_conv_tile(d, 1) >= 64),
               "the quantizer clip is folded into a bf16 BN+ReLU reduction on an LDS-DMA tile");
  RN_CHECK_ARG(d && dy && w_crsk && (dx || (part && !add_src)), "null argument");
  RN_CHECK_ARG(dx || rn_conv_tile(d, 1) >= 128, "a reduction-only dgrad (dx = NULL) needs the 224/256-row tile");
  if (gd_direct_ok(d, 1)) {
    RN_CHECK_ARG(dx, "grouped direct data gradient: dx required");
    if (!part) return gd_launch(d, 1, dy, w_crsk, dx, add_src, as_stream(stream));
    RN_CHECK_ARG(bn_x && bn_mean && bn_scale && bn_shift, "BN reduction needs x, mean, scale, shift");
    GdArgs r{};
    r.bnred = part; r.bn_x = (const bf16_t*)bn_x; r.bn_mean = bn_mean; r.bn_sc = bn_scale; r.bn_sh = bn_shift;
    r.bn_relu = relu;
    return gd_launch(d, 1, dy, w_crsk, dx, add_src, as_stream(stream), &r);
  }
  if (band_ok(d) && !part && !add_src && !clip && dx) return band_launch(d, dy, w_crsk, dx, 1, as_stream(stream));
  // (with the BN reduction only: the plain form -- epilogue 0, kept in the kernel for tests -- measured slower
  // than the tiles, 121.8 -> 182.4 us on stage 1's shape, profiles/r06/ab_dgrad_stream)
  if (part && d1_stream_ok(d, clip)) {
    RN_CHECK_ARG(bn_x && bn_mean && bn_scale && bn_shift, "BN reduction needs x, mean, scale, shift");
    return d1_stream_launch(d, 2, dy, w_crsk, dx, add_src, bn_x, bn_mean, nullptr, bn_scale, bn_shift, relu, part,
                            as_stream(stream));
  }
  IgemmArgs a = make_igemm_args(d, 1);
  a.x = dy; a.w = w_crsk; a.y = dx; a.add = add_src; a.bias = nullptr;
  if (part) {
    RN_CHECK_ARG(bn_x && bn_mean && bn_scale && bn_shift, "BN reduction needs x, mean, scale, shift");
    RN_CHECK_ARG(d->c % 8 == 0 && d->c == d->c_real, "BN reduction needs whole 8-channel chunks");
    int maxMc = 0;
    for (int z = 0; z < a.ncls; ++z) maxMc = std::max(maxMc, a.N * a.cls[z].Pc * a.cls[z].Qc);
    a.bnred = part; a.bn_x = bn_x; a.bn_mean = bn_mean; a.bn_sc = bn_scale; a.bn_sh = bn_shift;
    a.bn_relu = relu; a.bn_clip = clip; a.mt_max = (int)ceil_div(maxMc, 128);
  }
  hipStream_t st = as_stream(stream);
  if (d->dtype == RN_BF16) return launch_igemm<bf16_t, bf16_t>(a, st);
  return launch_igemm<float, float>(a, st);
}

int rn_conv_bwd_data_bnred_clip2(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                                 const void* other, const void* bn_x, const float* bn_mean, const float* bn_scale,
                                 const float* bn_shift, const float* clip, const float* clip2, float* part,
                                 rn_stream_t stream) {
  RN_CHECK_ARG(d && dy && w_crsk && dx && other && bn_x && bn_mean && bn_scale && bn_shift && clip && clip2 && part,
               "null argument");
  RN_CHECK_ARG(d->dtype == RN_BF16 && d->groups <= 1 && d->c % 8 == 0 && d->c == d->c_real && rn_conv_tile(d, 1) >= 64,
               "a quantizer pair's clips fold into a bf16 BN+ReLU reduction on an LDS-DMA tile");
  IgemmArgs a = make_igemm_args(d, 1);
  a.x = dy; a.w = w_crsk; a.y = dx; a.add = other; a.bias = nullptr;
  int maxMc = 0;
  for (int z = 0; z < a.ncls; ++z) maxMc = std::max(maxMc, a.N * a.cls[z].Pc * a.cls[z].Qc);
  a.bnred = part; a.bn_x = bn_x; a.bn_mean = bn_mean; a.bn_sc = bn_scale; a.bn_sh = bn_shift;
  a.bn_relu = 1; a.bn_clip = clip; a.bn_clip2 = clip2; a.mt_max = (int)ceil_div(maxMc, 128);
  return launch_igemm<bf16_t, bf16_t>(a, as_stream(stream));
}

int rn_conv_bwd_data_bnapply(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                             const void* add_src, const void* bn_x, const float* coef, const float* bn_scale,
                             const float* bn_shift, int32_t relu, rn_stream_t stream) {
  RN_CHECK_ARG(d && dy && w_crsk && dx && bn_x && coef && bn_scale && bn_shift, "null argument");
  RN_CHECK_ARG(d->dtype == RN_BF16 && d->c % 8 == 0 && d->c == d->c_real, "bf16, whole 8-channel chunks");
  RN_CHECK_ARG(rn_conv_tile(d, 1) >= 128, "BatchNorm-backward-apply dgrad needs the 224/256-row tile");
  if (d1_stream_ok(d, nullptr))
    return d1_stream_launch(d, 3, dy, w_crsk, dx, add_src, bn_x, nullptr, coef, bn_scale, bn_shift, relu, nullptr,
                            as_stream(stream));
  IgemmArgs a = make_igemm_args(d, 1);
  a.x = dy; a.w = w_crsk; a.y = dx; a.add = add_src; a.bias = nullptr;
  a.bn_x = bn_x; a.bn_coef = coef; a.bn_sc = bn_scale; a.bn_sh = bn_shift; a.bn_relu = relu;
  return launch_igemm<bf16_t, bf16_t>(a, as_stream(stream));
}

int rn_conv_bwd_data(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx, const void* add_src,
                     rn_stream_t stream) {
  return rn_conv_bwd_data_bnred(d, dy, w_crsk, dx, add_src, nullptr, nullptr, nullptr, nullptr, 0, nullptr, stream);
}

}  // extern "C"

namespace {
// The weight-gradient kernel choice for d. launch == false: only *ws_need (bytes of split-M partial
// slabs the chosen kernel stores when given a workspace; 0 = it adds into dw with atomics).
// i8: x holds int8 codes, dW = *xunit * sum dy * code (the streaming kernel and the 128 / 256-column
// LDS-DMA tiles only: rn_conv_wgrad_i8_supported)
int wgrad_dispatch(const rn_conv_desc* d, const void* x, const void* dy, float* dw, const float* in_scale,
                   const float* in_shift, float* ws, int64_t ws_bytes, int64_t* ws_need, bool launch,
                   hipStream_t st, const float* xunit = nullptr, bool i8 = false) {
  if (ws_need) *ws_need = 0;
  RN_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "in_scale / in_shift must both be set");
  RN_CHECK_ARG(!in_scale || d->groups == 1, "input transform on a grouped conv");
  RN_CHECK_ARG(!i8 || (!in_scale && d->dtype == RN_BF16 && d->groups <= 1 && d->c_real == d->c && d->c % 16 == 0),
               "int8 input codes: bf16 dy, dense, whole 16-channel chunks, no input transform");

  WgradArgs a{};
  a.x = x; a.dy = dy; a.dw = dw;
  a.in_sc = in_scale; a.in_sh = in_shift;
  a.xunit = xunit;
  a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.P = d->p; a.Q = d->q; a.K = d->k;
  a.ldy = d->k_pad; a.R = d->r; a.S = d->s; a.sh = d->stride_h; a.sw = d->stride_w;
  a.ph = d->pad_h; a.pw = d->pad_w;
  a.ncol_load = d->r * d->s * d->c;
  a.ncol = d->r * d->s * d->c_real;
  a.ldw = a.ncol;
  a.cblk = d->c;
  a.creal = d->c_real;
  const bool grouped = d->groups > 1;
  if (grouped) {
    a.grouped = 1;
    a.gk = d->k / d->groups; a.gc = d->c / d->groups;
    a.cblk = group_blk(a.gk, a.gc);
    a.ncol_load = d->r * d->s * a.cblk;
    a.ncol = d->r * d->s * a.gc;
    a.ldw = a.ncol;
    if (d->dtype == RN_BF16 && a.gk == a.gc && a.gk <= 32 && a.cblk == 64 && RN_GROUP_BLOCK == 64 &&
        g_tune[RN_TUNE_WGRAD_GD] != 1)
      a.gdiag = a.gk > 16 ? 2 : 1, a.gspread = g_tune[RN_TUNE_WGRAD_GD] != 2;
  }
  a.M = d->n * d->p * d->q;
  // (wgrad_big_kernel) buffer descriptor sizes; its launches need both < 2^31 elements (checked below)
  a.x_bytes = (int)(uint32_t)std::min<int64_t>((int64_t)d->n * d->h * d->w * d->c * (i8 ? 1 : 2), 0xFFFFFFFFll);
  a.dy_bytes = (int)(uint32_t)std::min<int64_t>((int64_t)a.M * a.ldy * 2, 0xFFFFFFFFll);
  // 1x1 / stride 1 / pad 0: x's row m is the gathered row m (wgrad_big_kernel DIR)
  const bool dir = d->r == 1 && d->s == 1 && d->stride_h == 1 && d->stride_w == 1 && d->pad_h == 0 &&
                   d->pad_w == 0 && d->c_real == d->c && d->groups <= 1;
  a.diag_noepi = g_tune[RN_TUNE_DIAG_WGRAD_NOEPI];
  a.fdQ = make_fastdiv(d->q); a.fdPQ = make_fastdiv(d->p * d->q);
  a.fdC = make_fastdiv(a.cblk); a.fdS = make_fastdiv(d->s);
  // split-M partial slabs (plain stores + wgrad_slab_reduce_kernel) instead of fp32 atomics: 2 x the
  // slab bytes at streaming rates vs the slab bytes at the chip's ~1.3 TB/s atomic rate
  // the BN+ReLU input transform runs on the LDS-DMA tiles for 1x1 convolutions (wgrad_big_kernel XF)
  const bool xf_big = !in_scale || (d->r == 1 && d->s == 1 && d->pad_h == 0 && d->pad_w == 0);
  // deterministic mode (rn_set_tuning 17): slabs for every kernel and dtype, never atomics
  const bool det = g_tune[RN_TUNE_DETERMINISTIC] == 1;
  // (the band kernels apply a 3x3 input transform too, with their slab)
  const bool band_xf = in_scale && d->r == 3 && d->s == 3 && d->pad_h == 1 && d->pad_w == 1 && d->stride_h == 1 &&
                       d->stride_w == 1;
  const bool slab_ok = det || (d->dtype == RN_BF16 && !grouped && (xf_big || band_xf) && d->c_real == d->c);
  if (det) a.gspread = 0;  // (grouped: each diagonal block on one wave, so one writer per element)
  auto finish = [&](int64_t split, const char* what) -> int {
    const int64_t need = slab_ok ? split * a.K * (int64_t)a.ldw * 4 : 0;
    if (ws_need) *ws_need = need;
    if (!launch) return 0;
    if (rn_check_launch(what)) return -1;
    if (a.slab) {
      const int64_t n = (int64_t)a.K * a.ldw;
      launch_slab_reduce(a.slab, (int)split, n, dw, st);
      return rn_check_launch("wgrad_slab_reduce");
    }
    return 0;
  };
  auto use_slab = [&](int64_t split) -> bool {
    const int64_t need = split * a.K * (int64_t)a.ldw * 4;
    a.slab = (slab_ok && ws && ws_bytes >= need) ? ws : nullptr;
    if (det && !a.slab) {
      rn_set_error("deterministic weight gradients need the split-M workspace (rn_conv_wgrad_ws_bytes)");
      return false;
    }
    return true;
  };
  // dense 3x3 / stride 1 / pad 1 with C = K in {64, 128, 256, 512} (every bottleneck conv2 but a stage's
  // first): image bands, dW slices per workgroup (wgrad_dband_kernel; rn_set_tuning 19 = 1: the tiled
  // kernels below). Needs the slab workspace.
  // (measured in isolation, tools/conv_bench.py: stage 1 89 vs 156 us on the tiled kernel; the 128 / 256 /
  // 512-channel forms lost to the 256-column tiled kernels -- 123 vs 106, 109 vs 76, 230 vs 80 us -- so
  // rn_set_tuning 19 = 2 is needed to run them)
  const int db = (d->c == 64 && d->w <= 62) ? 1 : g_tune[RN_TUNE_WGRAD_BAND] != 2 ? 0 :
                 (d->c == 128 && d->w <= 30) ? 2 : ((d->c == 256 || d->c == 512) && d->w <= 14) ? 3 : 0;
  if (!i8 && d->dtype == RN_BF16 && !grouped && db && d->r == 3 && d->s == 3 && d->stride_h == 1 &&
      d->stride_w == 1 && d->pad_h == 1 && d->pad_w == 1 && d->c_real == d->c && d->k == d->c &&
      d->k_pad == d->k && g_tune[RN_TUNE_WGRAD_BAND] != 1 && (int64_t)d->n * d->h * d->w * d->c < INT32_MAX) {
    DbArgs g{};
    g.x = (const bf16_t*)x; g.dy = (const bf16_t*)dy; g.N = d->n; g.H = d->h; g.W = d->w; g.C = d->c; g.K = d->k;
    g.in_sc = in_scale; g.in_sh = in_shift;
    const int cs = db == 1 ? 64 : 128, ks = db == 1 ? 64 : 32;
    const int slices = (d->c / cs) * (d->k / ks);
    const int64_t want = std::max<int64_t>(1, wgrad_cus() / slices);  // (the slab stays ~ CUs x slice)
    g.ipw = (int)ceil_div(d->n, std::min<int64_t>(d->n, want));
    const int64_t split = ceil_div(d->n, g.ipw);
    if (!launch) return finish(split, "wgrad_dband");
    if (ws && ws_bytes >= split * a.K * (int64_t)a.ldw * 4) {
      if (!use_slab(split)) return -1;
      g.slab = a.slab;
      const dim3 grid((unsigned)split, d->c / cs, d->k / ks);
#define RN_DBAND(XFV)                                                                                            \
  if (db == 1) hipLaunchKernelGGL((wgrad_dband_kernel<64, 64, 64, 2, 3, XFV>), grid, dim3(512), 0, st, g);     \
  else if (db == 2) hipLaunchKernelGGL((wgrad_dband_kernel<128, 32, 32, 1, 5, XFV>), grid, dim3(512), 0, st, g); \
  else hipLaunchKernelGGL((wgrad_dband_kernel<128, 32, 16, 2, 6, XFV>), grid, dim3(512), 0, st, g);
      if (in_scale) {
        RN_DBAND(1)
      } else {
        RN_DBAND(0)
      }
#undef RN_DBAND
      return finish(split, "wgrad_dband");
    }
  }
  // grouped 3x3 / stride 1 / pad 1 with 4 / 8 / 16 channels per group (ResNeXt stages 1-3, C = 128 /
  // 256 / 512): the whole block-diagonal dW per workgroup and channel slice (wgrad_gband_kernel;
  // rn_set_tuning 19 = 1: off)
  const int gb = (d->c == 128 && d->w <= 62) ? 1 : (d->c == 256 && d->w <= 30) ? 2 : (d->c == 512 && d->w <= 14) ? 3 : 0;
  if (d->dtype == RN_BF16 && grouped && gb && d->groups == 32 && d->r == 3 && d->s == 3 && d->stride_h == 1 &&
      d->stride_w == 1 && d->pad_h == 1 && d->pad_w == 1 && d->c == d->k && d->c == d->c_real &&
      g_tune[RN_TUNE_WGRAD_BAND] != 1 && (int64_t)d->n * d->h * d->w * d->c < INT32_MAX) {
    GbArgs g{};
    g.x = (const bf16_t*)x; g.dy = (const bf16_t*)dy; g.N = d->n; g.H = d->h; g.W = d->w; g.C = d->c;
    const int slices = gb == 3 ? 2 : 1;
    // (rn_set_tuning 23: these kernels' own percent of the chip, 0 = key 21's)
    const int gcus = g_tune[RN_TUNE_GBAND_SPLIT] > 0 ? std::max(8, chip_cus() * g_tune[RN_TUNE_GBAND_SPLIT] / 100)
                                                   : wgrad_cus();
    g.ipw = (int)std::max<int64_t>(1, ceil_div((int64_t)d->n * slices, gcus));
    const int64_t split = ceil_div(d->n, g.ipw);
    const int64_t need = split * a.K * (int64_t)a.ldw * 4;  // (a.ldw = 9 * channels per group)
    if (ws_need) *ws_need = need;
    if (!launch) return 0;
    if (ws && ws_bytes >= need) {
      g.slab = a.slab = ws;
      const dim3 grid((unsigned)split, slices);
      if (gb == 1) hipLaunchKernelGGL((wgrad_gband_kernel<128, 4, 64, 1, 2>), grid, dim3(512), 0, st, g);
      else if (gb == 2) hipLaunchKernelGGL((wgrad_gband_kernel<256, 8, 32, 1, 2>), grid, dim3(512), 0, st, g);
      else hipLaunchKernelGGL((wgrad_gband_kernel<256, 16, 16, 2, 2>), grid, dim3(512), 0, st, g);
      if (rn_check_launch("wgrad_gband")) return -1;
      const int64_t n = (int64_t)a.K * a.ldw;
      launch_slab_reduce(a.slab, (int)split, n, dw, st);
      return rn_check_launch("wgrad_slab_reduce");
    }
    if (ws_need) *ws_need = 0;
  }
  // 1x1 / stride 1 with the whole dW in one workgroup (K, C in {64, 128, 256}, K x C <= 32768): one
  // streaming pass over M per workgroup (wgrad_stream_kernel; rn_set_tuning 19 = 1: off)
  const bool one = d->r == 1 && d->s == 1 && d->stride_h == 1 && d->stride_w == 1 && d->pad_h == 0 && d->pad_w == 0;
  auto pw2 = [](int v) { return v == 64 || v == 128 || v == 256; };
  if (d->dtype == RN_BF16 && !grouped && one && pw2(d->k) && pw2(d->c) && d->k * d->c <= 32768 &&
      d->c_real == d->c && d->k_pad == d->k && g_tune[RN_TUNE_WGRAD_BAND] != 1 &&
      (int64_t)a.M * (d->k + d->c) * 2 < INT32_MAX) {
    const int64_t mtiles = ceil_div(a.M, 64);
    int64_t split = std::min<int64_t>(wgrad_cus(), std::max<int64_t>(1, mtiles / 4));
    // (at launch: no more splits than the workspace holds -- rn_set_tuning 21 may have changed since the
    // plan sized it, and the int8-codes form has no other kernel to fall back to)
    const int64_t slab1 = (int64_t)a.K * a.ldw * 4;
    if (launch && ws && ws_bytes >= slab1) split = std::min<int64_t>(split, ws_bytes / slab1);
    a.m_per_split = (int)(ceil_div(mtiles, split) * 64);
    const int64_t nsplit = ceil_div(a.M, a.m_per_split);
    if (!launch) return finish(nsplit, "wgrad_stream");
    if (ws && ws_bytes >= nsplit * a.K * (int64_t)a.ldw * 4) {
      if (!use_slab(nsplit)) return -1;
      const dim3 grid((unsigned)nsplit);
      const bool t = in_scale != nullptr;
#define RN_STREAM(KK, CC)                                                                         \
  if (d->k == KK && d->c == CC) {                                                                 \
    if (t) hipLaunchKernelGGL((wgrad_stream_kernel<KK, CC, 1, 3>), grid, dim3(512), 0, st, a);    \
    else if (i8) hipLaunchKernelGGL((wgrad_stream_kernel<KK, CC, 0, 3, 1>), grid, dim3(512), 0, st, a); \
    else hipLaunchKernelGGL((wgrad_stream_kernel<KK, CC, 0, 3>), grid, dim3(512), 0, st, a);      \
  }
      RN_STREAM(64, 64) RN_STREAM(64, 128) RN_STREAM(64, 256) RN_STREAM(128, 64) RN_STREAM(128, 128)
      RN_STREAM(128, 256) RN_STREAM(256, 64) RN_STREAM(256, 128)
#undef RN_STREAM
      return finish(nsplit, "wgrad_stream");
    }
  }
  // 256-column, 8-wave LDS-DMA tiles (rn_set_tuning 5: 1 = on, default off) for dense bf16 layers
  // with >= 128 output channels and >= 256 columns; the M range is split so that the grid is one
  // round of one workgroup per CU, with >= 4 M-tiles per workgroup. Measured slower than the
  // 128-tile kernel on every ResNet-50 layer: with the M split, the fp32 atomic epilogue issues
  // (workgroups x tile area) adds, 4x more per workgroup at 256x256, and that dominates the
  // small-M layers (stage 3-4).
  // (default for the stem's padded channels, c_real < c = 8; rn_set_tuning 5 = 4 for every 64-channel layer)
  const bool stem_dma = d->c_real < d->c && d->c == 8 && g_tune[RN_TUNE_WGRAD_BIG] != 3;
  if (!i8 && d->dtype == RN_BF16 && !grouped && !in_scale && (d->c_real == d->c || stem_dma) && a.K <= 64 &&
      a.ncol_load > 64 && (g_tune[RN_TUNE_WGRAD_BIG] == 4 || stem_dma) &&
      (int64_t)d->n * d->h * d->w * d->c < INT32_MAX && (int64_t)a.M * a.ldy < INT32_MAX) {
    // 64 x 128 LDS-DMA tiles for the 64-channel layers (4 waves, 3 buffers, two workgroups per CU)
    a.nct = (int)ceil_div(a.ncol_load, 128);
    a.nkt = 1;
    const int64_t tiles = a.nct;
    const int64_t mtiles = ceil_div(a.M, 64);
    int64_t split = std::min<int64_t>(std::max<int64_t>(1, 512 / tiles), std::max<int64_t>(1, mtiles / 8));
    a.m_per_split = (int)(ceil_div(mtiles, split) * 64);
    split = ceil_div(a.M, a.m_per_split);
    if (!launch) return finish(split, "wgrad_dma64");
    if (!use_slab(split)) return -1;
    hipLaunchKernelGGL((wgrad_big_kernel<64, 3, 128>), dim3((unsigned)(tiles * split)), dim3(256), 0, st, a);
    return finish(split, "wgrad_dma64");
  }
  // with a slab workspace (rn_conv_bwd_filter_ws) the 256-column 8-wave tiles below are the default
  // for >= 128 output channels and >= 256 columns: their main loop is the faster one, and the
  // 4x larger per-workgroup tile no longer costs atomics
  const bool big256 = (g_tune[RN_TUNE_WGRAD_BIG] == 1 || (g_tune[RN_TUNE_WGRAD_BIG] == 0 && slab_ok && ws)) &&
                      d->dtype == RN_BF16 && !grouped && xf_big && d->c_real == d->c && a.K >= 128 &&
                      a.ncol_load >= 256 && (int64_t)d->n * d->h * d->w * d->c < INT32_MAX &&
                      (int64_t)a.M * a.ldy < INT32_MAX;
  if (d->dtype == RN_BF16 && !grouped && xf_big && d->c_real == d->c && !big256 &&
      (g_tune[RN_TUNE_WGRAD_BIG] == 0 || g_tune[RN_TUNE_WGRAD_BIG] == 2 || g_tune[RN_TUNE_WGRAD_BIG] == 4) &&
      a.K > 64 && a.ncol_load > 64 && (int64_t)d->n * d->h * d->w * d->c < INT32_MAX &&
      (int64_t)a.M * a.ldy < INT32_MAX) {
    // 128 x 128 LDS-DMA tiles, 4 waves, two workgroups per CU (default; measured -0.4 % step time
    // over the register-staged wgrad_kernel, which rn_set_tuning 5 = 3 selects). The M split targets
    // rn_set_tuning 2 workgroups per CU (default 2): every workgroup adds its tile into dw with
    // fp32 atomics, so the atomic traffic is (workgroups x 64 KB).
    a.nct = (int)ceil_div(a.ncol_load, 128);
    a.nkt = (int)ceil_div(a.K, 128);
    const int64_t tiles = (int64_t)a.nct * a.nkt;
    const int64_t mtiles = ceil_div(a.M, 64);
    const int64_t target = wgrad_cus() * (g_tune[RN_TUNE_WGRAD_BLOCKS_PER_CU] > 0 ? g_tune[RN_TUNE_WGRAD_BLOCKS_PER_CU] : 2);
    int64_t split = std::min<int64_t>(std::max<int64_t>(1, target / tiles), std::max<int64_t>(1, mtiles / 8));
    a.m_per_split = (int)(ceil_div(mtiles, split) * 64);
    split = ceil_div(a.M, a.m_per_split);
    if (!launch) return finish(split, "wgrad_dma128");
    if (!use_slab(split)) return -1;
    const dim3 g128((unsigned)(tiles * split));
#define RN_W128(DV)                                                                                        \
  if (in_scale) hipLaunchKernelGGL((wgrad_big_kernel<128, 2, 128, 1, 0, DV>), g128, dim3(256), 0, st, a);   \
  else if (i8) hipLaunchKernelGGL((wgrad_big_kernel<128, 2, 128, 0, 1, DV>), g128, dim3(256), 0, st, a);    \
  else hipLaunchKernelGGL((wgrad_big_kernel<128, 2, 128, 0, 0, DV>), g128, dim3(256), 0, st, a);
    if (dir) {
      RN_W128(1)
    } else {
      RN_W128(0)
    }
#undef RN_W128
    return finish(split, "wgrad_dma128");
  }
  if (big256) {
    const int bmk = a.K >= 256 ? 256 : 128;
    a.nct = (int)ceil_div(a.ncol_load, 256);
    a.nkt = (int)ceil_div(a.K, bmk);
    const int64_t tiles = (int64_t)a.nct * a.nkt;
    const int64_t mtiles = ceil_div(a.M, 64);
    int64_t split = std::min<int64_t>(std::max<int64_t>(1, wgrad_cus() / tiles), std::max<int64_t>(1, mtiles / 4));
    a.m_per_split = (int)(ceil_div(mtiles, split) * 64);
    split = ceil_div(a.M, a.m_per_split);
    if (!launch) return finish(split, "wgrad_big");
    if (!use_slab(split)) return -1;
    dim3 grid((unsigned)(tiles * split));
#define RN_W256(DV)                                                                                              \
  if (in_scale) {                                                                                               \
    if (bmk == 256) hipLaunchKernelGGL((wgrad_big_kernel<256, 2, 256, 1, 0, DV>), grid, dim3(512), 0, st, a);    \
    else hipLaunchKernelGGL((wgrad_big_kernel<128, 3, 256, 1, 0, DV>), grid, dim3(512), 0, st, a);               \
  } else if (i8) {                                                                                              \
    if (bmk == 256) hipLaunchKernelGGL((wgrad_big_kernel<256, 2, 256, 0, 1, DV>), grid, dim3(512), 0, st, a);    \
    else hipLaunchKernelGGL((wgrad_big_kernel<128, 3, 256, 0, 1, DV>), grid, dim3(512), 0, st, a);               \
  } else if (bmk == 256) hipLaunchKernelGGL((wgrad_big_kernel<256, 2, 256, 0, 0, DV>), grid, dim3(512), 0, st, a); \
  else hipLaunchKernelGGL((wgrad_big_kernel<128, 3, 256, 0, 0, DV>), grid, dim3(512), 0, st, a);
    if (dir) {
      RN_W256(1)
    } else {
      RN_W256(0)
    }
#undef RN_W256
    return finish(split, "wgrad_big");
  }
  if (i8) {  // (a plan-time query, launch == false, sets no error)
    if (launch) rn_set_error("int8 input codes: no weight-gradient kernel for this shape (rn_conv_wgrad_i8_supported)");
    return -1;
  }
  // 64-wide tiles where K or the column count is <= 64 (stage-1 layers): a 128 tile would spend
  // half (or three quarters) of its MFMAs on zero rows / columns
  const int bmk = (grouped || a.K <= 64) ? 64 : 128;
  const int bnc = (grouped || a.ncol_load <= 64) ? 64 : 128;
  const int tiles = (int)(ceil_div(a.ncol_load, bnc) * ceil_div(a.K, bmk));
  const int bkm = d->dtype == RN_BF16 ? 64 : 32;
  const int64_t mstages = ceil_div(a.M, bkm);
  // split M so that the whole grid is ONE round of resident blocks (floor: a partly filled second
  // round of long blocks is the worst tail), with >= 8 stages per block. Resident blocks per CU
  // of each tile variant (VGPR / LDS bound): 128x128 -> 2, 64x128 / 128x64 -> 3, 64x64 -> 5.
  // (the bf16 grouped block-diagonal-skip kernel (gdiag): 8, measured on the ResNeXt-50 3x3 layers --
  // 2.08 vs 2.39 ms per step at 5, 2.23 at 3, 2.20 at 12; tools/runs/gsplit.sh. Other grouped
  // variants keep the 64x64 tile's 5.) The chip size is chip_cus(): the device's CU count, cached
  // once per process (rn_conv_wgrad_ws_bytes sizes the slab workspace from this same split at plan
  // time, and the launch agrees with it), 256 on a host without a GPU (plan-only dry runs).
  const int kSplitCus = wgrad_cus();
  int per_cu = (grouped && a.gdiag) ? 8 : (bmk == 128 && bnc == 128) ? 2 : (bmk == 64 && bnc == 64) ? (in_scale ? 4 : 5) : 3;
  if (g_tune[RN_TUNE_WGRAD_BLOCKS_PER_CU] > 0) per_cu = g_tune[RN_TUNE_WGRAD_BLOCKS_PER_CU];
  int64_t want = std::max<int64_t>(1, (int64_t)per_cu * kSplitCus / tiles);
  int64_t maxsplit = std::max<int64_t>(1, mstages / 8);
  int64_t split = std::min(want, maxsplit);
  int64_t stages_per = ceil_div(mstages, split);
  a.m_per_split = (int)(stages_per * bkm);
  split = ceil_div(a.M, a.m_per_split);
  a.nct = (int)ceil_div(a.ncol_load, bnc);
  a.nkt = (int)ceil_div(a.K, bmk);
  dim3 grid((unsigned)(a.nct * a.nkt * split));
  if (det) {  // this register-staged kernel stores slabs only in the deterministic mode
    if (!launch) return finish(split, "wgrad");
    if (!use_slab(split)) return -1;
  } else {
    if (ws_need) *ws_need = 0;
    if (!launch) return 0;
    a.slab = nullptr;
  }
  if (grouped) {
    if (d->dtype == RN_BF16 && a.gdiag)
      hipLaunchKernelGGL((wgrad_kernel<bf16_t, RN_GROUP_BLOCK, RN_GROUP_BLOCK, false, true>), grid, dim3(256), 0, st, a);
    else if (d->dtype == RN_BF16)
      hipLaunchKernelGGL((wgrad_kernel<bf16_t, RN_GROUP_BLOCK, RN_GROUP_BLOCK>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((wgrad_kernel<float, RN_GROUP_BLOCK, RN_GROUP_BLOCK>), grid, dim3(256), 0, st, a);
  } else if (d->dtype == RN_BF16) {
    if (in_scale) launch_wgrad_tiles<bf16_t, true>(bmk, bnc, grid, st, a);
    else launch_wgrad_tiles<bf16_t, false>(bmk, bnc, grid, st, a);
  } else {
    if (in_scale) launch_wgrad_tiles<float, true>(bmk, bnc, grid, st, a);
    else launch_wgrad_tiles<float, false>(bmk, bnc, grid, st, a);
  }
  if (det) return finish(split, "wgrad");
  return rn_check_launch("wgrad");
}
}  // namespace

extern "C" {

int rn_conv_bwd_filter_x(const rn_conv_desc* d, const void* x, const void* dy, float* dw, const float* in_scale,
                         const float* in_shift, void* ws, int64_t ws_bytes, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && dy && dw, "null argument");
  RN_CHECK_ARG(ws_bytes >= 0 && (ws || ws_bytes == 0), "bad workspace");
  RN_CHECK_ARG(((uintptr_t)ws & 15) == 0, "workspace must be 16-byte aligned");
  return wgrad_dispatch(d, x, dy, dw, in_scale, in_shift, reinterpret_cast<float*>(ws), ws_bytes, nullptr, true,
                        as_stream(stream));
}

int64_t rn_conv_wgrad_ws_bytes(const rn_conv_desc* d) {
  if (!d) return -1;
  int64_t need = 0;
  if (wgrad_dispatch(d, nullptr, nullptr, nullptr, nullptr, nullptr, reinterpret_cast<float*>(16), INT64_MAX, &need,
                     false, nullptr))
    return -1;
  return need;
}

int rn_conv_bwd_filter_ws(const rn_conv_desc* d, const void* x, const void* dy, float* dw, void* ws, int64_t ws_bytes,
                          rn_stream_t stream) {
  RN_CHECK_ARG(d && x && dy && dw, "null argument");
  RN_CHECK_ARG(ws_bytes >= 0 && (ws || ws_bytes == 0), "bad workspace");
  RN_CHECK_ARG(((uintptr_t)ws & 15) == 0, "workspace must be 16-byte aligned");
  return wgrad_dispatch(d, x, dy, dw, nullptr, nullptr, reinterpret_cast<float*>(ws), ws_bytes, nullptr, true,
                        as_stream(stream));
}

int rn_conv_bwd_filter(const rn_conv_desc* d, const void* x, const void* dy, float* dw, rn_stream_t stream) {
  return rn_conv_bwd_filter_x(d, x, dy, dw, nullptr, nullptr, nullptr, 0, stream);
}

int32_t rn_conv_wgrad_i8_supported(const rn_conv_desc* d) {
  if (!d || d->dtype != RN_BF16 || d->groups > 1 || d->c_real != d->c || d->c % 16 != 0) return 0;
  int64_t need = 0;
  const int r = wgrad_dispatch(d, nullptr, nullptr, nullptr, nullptr, nullptr, reinterpret_cast<float*>(16), INT64_MAX,
                               &need, false, nullptr, nullptr, true);
  return r == 0 && need > 0 ? 1 : 0;
}

int64_t rn_conv_wgrad_i8_ws_bytes(const rn_conv_desc* d) {
  if (!rn_conv_wgrad_i8_supported(d)) return -1;
  int64_t need = 0;
  if (wgrad_dispatch(d, nullptr, nullptr, nullptr, nullptr, nullptr, reinterpret_cast<float*>(16), INT64_MAX, &need,
                     false, nullptr, nullptr, true))
    return -1;
  return need;
}

int rn_conv_bwd_filter_i8(const rn_conv_desc* d, const void* x_codes, const float* x_unit, const void* dy, float* dw,
                          void* ws, int64_t ws_bytes, rn_stream_t stream) {
  RN_CHECK_ARG(d && x_codes && x_unit && dy && dw, "null argument");
  RN_CHECK_ARG(ws_bytes >= 0 && (ws || ws_bytes == 0), "bad workspace");
  RN_CHECK_ARG(((uintptr_t)ws & 15) == 0, "workspace must be 16-byte aligned");
  RN_CHECK_ARG(rn_conv_wgrad_i8_supported(d), "int8 input codes: unsupported shape (rn_conv_wgrad_i8_supported)");
  return wgrad_dispatch(d, x_codes, dy, dw, nullptr, nullptr, reinterpret_cast<float*>(ws), ws_bytes, nullptr, true,
                        as_stream(stream), x_unit, true);
}

// ---------------------------------------------------------------- stem over the padded NHWC4 image
namespace {
// The stem convolution (conv0: 7x7 / stride 2 over bn_data's output, symbol/resnet.py:90-93) over image
// bands, as conv3x3c64_band_kernel does for stage 1's 3x3 layers. On the implicit-GEMM tile every output
// row DMAs its 8 x 8 x 4 input patch on its own (a gather of 32 16-byte pieces per row, whose issue bounds
// the launch: 198 us for a 411 MB output); here a band of 4 output rows takes its 14 input rows in one
// contiguous DMA (the zero-bordered image needs no bounds), and every MFMA B fragment is one 16-byte LDS
// read: k-step r (kernel row r, 32 k = taps s 0..7 x 4 channels), lane (q, c) supplies taps 2q, 2q + 1 of
// output pixel c = input pixels 2 col + 2q, + 1, adjacent in the band row. The 64 x 256 weights stay in
// LDS (rows XOR-swizzled by 16-byte chunk: the 16 lanes of a channel block read 16 distinct chunks). Seven
// waves, wave w = 16-pixel blocks 4w..4w + 3 of the band's 4 Q <= 448 pixels, all 64 channels; operands
// swapped so a lane's accumulator is 4 consecutive channels of one pixel (8-byte stores).
struct StemBandArgs {
  const void* x4;  // [N][hp][wp][4] bf16, zero-bordered
  const void* w4;  // [64][8][8][4] bf16
  void* y;         // [N][P][Q][64] bf16
  float* part;     // (STATS) [workgroup][S1 | S2 | pivot][64]: bn0's statistics of the stored y, one block per
                   // workgroup (its bands' rows, the same count for every workgroup), pivot = its first pixel
  int N, P, Q, hp, wp, pb, nbands, x_bytes, y_bytes;
};
constexpr int kStemInRows = 14;                  // 4 output rows at stride 2 + the 8-row kernel window - 2
constexpr int kStemBandBytes = 26 * 1024;        // 26 whole 64-lane DMA instructions >= 14 rows x 232 px x 8 B
__global__ __launch_bounds__(448, 1) void stem_band_kernel(StemBandArgs p) {
  const bool STATS = p.part != nullptr;  // (a runtime switch: this kernel has C linkage, no template)
  // 84 KB: two band buffers, the weights; (STATS) the 7 waves' sums and the pivots
  __shared__ __attribute__((aligned(16))) uint4 smem[(2 * kStemBandBytes + 64 * 512 + 7 * 64 * 8 + 64 * 4) / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const v4i rs_x = make_rsrc(p.x4, (uint32_t)p.x_bytes);
  const v4i rs_w = make_rsrc(p.w4, 64 * 512);
  const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.y_bytes, 0x00020000);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  constexpr uint32_t kW = 2 * kStemBandBytes;
  // the weights: 2048 chunks (channel o, phys chunk f) over waves 0-3, f holding logical chunk f ^ (o & 15)
  if (wid < 4) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ins = wid * 8 + j, chunk = ins * 64 + lane;
      const int o = chunk >> 5, logical = (chunk & 31) ^ (o & 15);
      dma16_asm(rs_w, lds0 + kW + ins * 1024, (uint32_t)((o * 256 + logical * 8) * 2));
    }
  }
  // band b -> buffer bb: the 14 input rows from 2 p0 are one contiguous range of the image (26 pieces over
  // waves 0-6); pieces past the image's last row read zeros
  const uint32_t img_bytes = (uint32_t)p.hp * p.wp * 8;
  auto issue_band = [&](int b, int bb) __attribute__((always_inline)) {
    const int n = b / p.pb, p0 = (b - n * p.pb) * 4;
    const uint32_t off0 = (uint32_t)(2 * p0) * p.wp * 8;
    for (int ins = wid; ins < 26; ins += 7) {
      const uint32_t off = off0 + (uint32_t)(ins * 64 + lane) * 16;
      dma16_asm(rs_x, lds0 + bb * kStemBandBytes + ins * 1024, off < img_bytes ? (uint32_t)n * img_bytes + off : kOob);
    }
  };
  // this lane's output pixels pp = (4 wid + i) 16 + c of the band = (orow, ocol); k-step r reads the band at
  // byte ab[i] + r * wp * 8 (the 16 bytes of input pixels 2 ocol + 2q, + 1 of row 2 orow + r); channel block
  // j's weights at wb[j] + chunk (4 r + q) ^ (o & 15)
  const int q = lane >> 4, c = lane & 15;
  int ab[4], orow[4], ocol[4], pp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pp[i] = (4 * wid + i) * 16 + c;
    orow[i] = min(pp[i] / p.Q, 3);
    ocol[i] = min(pp[i] - orow[i] * p.Q, p.Q - 1);
    ab[i] = ((2 * orow[i]) * (p.wp >> 1) + ocol[i] + q) * 16;
  }
  int wb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wb[j] = (int)kW + (16 * j + c) * 512;
  const int rowb = p.wp * 8;
  const char* lds = reinterpret_cast<const char*>(smem);
  float* red = reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + kW + 64 * 512);  // [wave][64][2]
  float* piv = red + 7 * 64 * 2;                                                         // [64]
  // (STATS) this lane's shifted sums of channels 16 j + 4 q + e (k = 4 j + e) over its valid pixels
  float s1[16], s2[16], pv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) s1[k] = s2[k] = pv[k] = 0.f;
  int it = 0;
  int b = blockIdx.x;
  if (b < p.nbands) issue_band(b, 0);
  for (; b < p.nbands; b += gridDim.x, ++it) {
    const int bb = it & 1;
    if (it == 0) wait_vmcnt<0>();
    else wait_vmcnt<16>();  // (the previous band's 16 stores may stay in flight)
    __syncthreads();        // the band has landed for every wave; every wave is done with the other buffer
    if (b + (int)gridDim.x < p.nbands) issue_band(b + gridDim.x, bb ^ 1);
    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    const int boff = bb * kStemBandBytes;
    uint4 fa[2][4], fb[2][4];
    auto ld = [&](int r, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[slot][i] = *reinterpret_cast<const uint4*>(lds + boff + ab[i] + r * rowb);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[slot][j] = *reinterpret_cast<const uint4*>(lds + wb[j] + (((4 * r + q) ^ c) << 4));
    };
    ld(0, 0);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (r + 1 < 8) ld(r + 1, (r + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);  // (hipcc otherwise sinks every read next to its MFMA)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_slab<bf16_t>(acc[i][j], fb[r & 1][j], fa[r & 1][i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int n = b / p.pb, p0 = (b - n * p.pb) * 4;
    if (STATS) {
      if (it == 0) {  // the pivots: the stored values of the workgroup's first pixel (wave 0, block 0, lane c = 0)
        if (wid == 0 && c == 0)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) piv[16 * j + 4 * q + e] = __uint_as_float((uint32_t)f2bf(acc[0][j][e]) << 16);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) pv[k] = piv[16 * (k >> 2) + 4 * q + (k & 3)];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = p0 + orow[i];
      const bool ok = pp[i] < 4 * p.Q && h < p.P;
      const int obase = (((n * p.P + h) * p.Q + ocol[i]) * 64 + 4 * q) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        const uint32_t voff = ok ? (uint32_t)(obase + j * 32) : 0x80000000u;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo, hi}, rs_y, voff, 0, 0);
        if (STATS) {  // on the stored (rounded) values, as a statistics pass would read them
          const uint32_t vw[4] = {lo << 16, lo & 0xFFFF0000u, hi << 16, hi & 0xFFFF0000u};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = 4 * j + e;
            const float dv = ok ? __uint_as_float(vw[e]) - pv[k] : 0.f;
            s1[k] += dv;
            s2[k] = fmaf(dv, dv, s2[k]);
          }
        }
      }
    }
  }
  if (STATS) {
    // the 16 pixel lanes of each channel quad (xor 1, 2, 4, 8), then the 7 waves in order through LDS
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        s1[k] += __shfl_xor(s1[k], o, 64);
        s2[k] += __shfl_xor(s2[k], o, 64);
      }
    if (c == 0)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int ch = 16 * (k >> 2) + 4 * q + (k & 3);
        red[(wid * 64 + ch) * 2] = s1[k];
        red[(wid * 64 + ch) * 2 + 1] = s2[k];
      }
    __syncthreads();
    if (tid < 64) {
      float a1 = red[tid * 2], a2 = red[tid * 2 + 1];
#pragma unroll
      for (int w = 1; w < 7; ++w) {
        a1 += red[(w * 64 + tid) * 2];
        a2 += red[(w * 64 + tid) * 2 + 1];
      }
      float* dst = p.part + (int64_t)blockIdx.x * 3 * 64 + tid;
      dst[0] = a1;
      dst[64] = a2;
      dst[128] = piv[tid];
    }
  }
}
// stem_band_kernel for this stem? (rn_set_tuning 26 = 1 or 2: the implicit-GEMM tile)
bool stem_band_ok(const rn_conv_desc* d, int32_t hp, int32_t wp) {
  return g_tune[RN_TUNE_CONV_BAND] == 0 && d->stride_h == 2 && d->stride_w == 2 && d->k == 64 && d->k_pad == 64 &&
         wp % 2 == 0 && wp <= 232 && d->q <= 112 && (int64_t)d->n * d->p * d->q * 64 * 2 < INT32_MAX;
}

bool stem_p4_ok(const rn_conv_desc* d, int32_t hp, int32_t wp) {
  return d && d->dtype == RN_BF16 && d->groups == 1 && d->c_real <= 4 && d->k <= 64 && d->r <= 8 && d->s <= 8 &&
         hp >= (d->p - 1) * d->stride_h + 8 && wp >= (d->q - 1) * d->stride_w + 8 &&
         (int64_t)d->n * hp * wp * 4 < INT32_MAX;
}
}  // namespace

__global__ void stem_pack_p4_kernel(const float* __restrict__ wm, bf16_t* __restrict__ out, int K, int R, int S,
                                    int creal) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // out[k][r<8][s<8][c<4]
  if (i >= K * 256) return;
  const int c = i & 3, s = (i >> 2) & 7, r = (i >> 5) & 7, k = i >> 8;
  const float v = (c < creal && s < S && r < R) ? wm[((int64_t)(k * R + r) * S + s) * creal + c] : 0.f;
  out[i] = f2bf(v);
}

int32_t rn_stem_p4_supported(const rn_conv_desc* d, int32_t hp, int32_t wp) { return stem_p4_ok(d, hp, wp) ? 1 : 0; }

int rn_stem_weight_pack_p4(const rn_conv_desc* d, const float* wm, void* w4, rn_stream_t stream) {
  RN_CHECK_ARG(d && wm && w4 && d->dtype == RN_BF16 && d->c_real <= 4 && d->r <= 8 && d->s <= 8, "bad arguments");
  hipLaunchKernelGGL(stem_pack_p4_kernel, dim3((d->k * 256 + 255) / 256), dim3(256), 0, as_stream(stream), wm,
                     (bf16_t*)w4, d->k, d->r, d->s, d->c_real);
  return rn_check_launch("stem_weight_pack_p4");
}

int64_t rn_stem_bnstats_blocks(const rn_conv_desc* d, int32_t hp, int32_t wp) {
  // the band kernel's workgroups when each takes the same number of whole bands (4 output rows each)
  if (!d || !stem_p4_ok(d, hp, wp) || !stem_band_ok(d, hp, wp) || d->p % 4) return 0;
  const int nb = d->n * (d->p / 4), g = chip_cus();
  return nb <= g ? nb : (nb % g == 0 ? g : 0);
}

int rn_stem_conv_fwd_p4(const rn_conv_desc* d, const void* x4, const void* w4, void* y, int32_t hp, int32_t wp,
                        rn_stream_t stream) {
  return rn_stem_conv_fwd_p4_bnstats(d, x4, w4, y, hp, wp, nullptr, stream);
}

int rn_stem_conv_fwd_p4_bnstats(const rn_conv_desc* d, const void* x4, const void* w4, void* y, int32_t hp,
                                int32_t wp, float* part, rn_stream_t stream) {
  RN_CHECK_ARG(x4 && w4 && y, "null argument");
  RN_CHECK_ARG(stem_p4_ok(d, hp, wp), "unsupported stem shape for the padded NHWC4 path");
  RN_CHECK_ARG(!part || rn_stem_bnstats_blocks(d, hp, wp) > 0,
               "the stem's BatchNorm statistics need the band kernel with whole bands per workgroup "
               "(rn_stem_bnstats_blocks)");
  if (stem_band_ok(d, hp, wp)) {
    StemBandArgs s{};
    s.x4 = x4; s.w4 = w4; s.y = y; s.part = part;
    s.N = d->n; s.P = d->p; s.Q = d->q; s.hp = hp; s.wp = wp; s.pb = (d->p + 3) / 4; s.nbands = d->n * s.pb;
    s.x_bytes = (int)((int64_t)d->n * hp * wp * 4 * 2);
    s.y_bytes = (int)((int64_t)d->n * d->p * d->q * 64 * 2);
    const dim3 grid((unsigned)std::min(s.nbands, chip_cus()));
    hipLaunchKernelGGL(stem_band_kernel, grid, dim3(448), 0, as_stream(stream), s);
    return rn_check_launch("stem_band");
  }
  IgemmArgs a{};
  a.x = x4; a.w = w4; a.y = y;
  a.N = d->n; a.H = hp; a.W = wp; a.C = 4; a.P = d->p; a.Q = d->q; a.K = d->k; a.ldo = d->k_pad;
  a.S = 8; a.wrow = 256; a.hmul = d->stride_h; a.wmul = d->stride_w;
  a.ostep_h = 1; a.ostep_w = 1; a.cblk = 4; a.gcol = 1 << 30; a.gred = 0;
  a.ncls = 1;
  IgemmCls& c = a.cls[0];
  c.Pc = d->p; c.Qc = d->q; c.nr = 1; c.ns = 1;
  c.fdQ = make_fastdiv(c.Qc); c.fdPQ = make_fastdiv(c.Pc * c.Qc);
  a.x_bytes = (int)((int64_t)d->n * hp * wp * 4 * 2);
  a.w_bytes = d->k * 256 * 2;
  a.sched = g_tune[RN_TUNE_IGEMM_SCHED];
  a.epi_sync = g_tune[RN_TUNE_EPI_SYNC];
  a.nt_store = (g_tune[RN_TUNE_BN_NT] & 16) != 0;
  a.ntn = 1;
  const int64_t M = (int64_t)d->n * d->p * d->q;
  hipLaunchKernelGGL((igemm_big_kernel<64, 2, 0, true, 256, 2>), dim3((unsigned)ceil_div(M, 256)), dim3(256), 0,
                     as_stream(stream), a);
  return rn_check_launch("stem_conv_fwd_p4");
}

int rn_stem_conv_wgrad_p4(const rn_conv_desc* d, const void* x4, const void* dy, float* dw, int32_t hp, int32_t wp,
                          rn_stream_t stream) {
  RN_CHECK_ARG(x4 && dy && dw, "null argument");
  RN_CHECK_ARG(stem_p4_ok(d, hp, wp), "unsupported stem shape for the padded NHWC4 path");
  RN_CHECK_ARG((int64_t)d->n * d->p * d->q * d->k_pad < INT32_MAX, "dy exceeds 2^31 elements");
  WgradArgs a{};
  a.x = x4; a.dy = dy; a.dw = dw;
  a.N = d->n; a.H = hp; a.W = wp; a.C = 4; a.P = d->p; a.Q = d->q; a.K = d->k;
  a.ldy = d->k_pad; a.R = d->r; a.S = d->s; a.sh = d->stride_h; a.sw = d->stride_w; a.ph = 0; a.pw = 0;
  a.ncol_load = 256;
  a.ncol = d->r * d->s * d->c_real;
  a.ldw = a.ncol;
  a.cblk = 4;
  a.creal = d->c_real;
  a.p4 = 1;
  a.M = d->n * d->p * d->q;
  a.fdQ = make_fastdiv(d->q); a.fdPQ = make_fastdiv(d->p * d->q);
  a.fdC = make_fastdiv(4); a.fdS = make_fastdiv(8);
  a.x_bytes = (int)((int64_t)d->n * hp * wp * 4 * 2);
  a.dy_bytes = (int)((int64_t)a.M * a.ldy * 2);
  a.nct = 2;
  a.nkt = 1;
  const int64_t tiles = a.nct;
  const int64_t mtiles = ceil_div(a.M, 64);
  int64_t split = std::min<int64_t>(std::max<int64_t>(1, 512 / tiles), std::max<int64_t>(1, mtiles / 8));
  a.m_per_split = (int)(ceil_div(mtiles, split) * 64);
  split = ceil_div(a.M, a.m_per_split);
  hipLaunchKernelGGL((wgrad_big_kernel<64, 3, 128>), dim3((unsigned)(tiles * split)), dim3(256), 0, as_stream(stream),
                     a);
  return rn_check_launch("stem_conv_wgrad_p4");
}

int rn_conv_weight_pack(const rn_conv_desc* d, const float* wm, void* w_krsc, void* w_crsk,
                        rn_stream_t stream) {
  RN_CHECK_ARG(d && wm, "null argument");
  hipStream_t st = as_stream(stream);
  const int RS = d->r * d->s;
  if (d->groups > 1) {
    const int cpg = d->c / d->groups, kpg = d->k / d->groups;
    for (int which = 0; which < 2; ++which) {
      void* out = which == 0 ? w_krsc : w_crsk;
      if (!out) continue;
      if (gd_direct_ok(d, which)) {
        hipLaunchKernelGGL(pack_group_direct_kernel, dim3(grid_for((int64_t)d->c * 9 * cpg)), dim3(256), 0, st, wm,
                           (bf16_t*)out, d->c, cpg, which);
        continue;
      }
      const int ncols = which == 0 ? d->k : d->c;
      const int gcol = which == 0 ? kpg : cpg, gred = which == 0 ? cpg : kpg;
      const int cblk = group_blk(gcol, gred);
      const int64_t total = (int64_t)ncols * RS * cblk;
      if (d->dtype == RN_BF16)
        hipLaunchKernelGGL(pack_group_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, wm, (bf16_t*)out,
                           ncols, RS, cblk, gcol, gred, cpg, which);
      else
        hipLaunchKernelGGL(pack_group_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, wm, (float*)out,
                           ncols, RS, cblk, gcol, gred, cpg, which);
    }
    return rn_check_launch("weight_pack");
  }
  if (w_krsc) {
    const int64_t total = (int64_t)d->k * RS * d->c;
    if (d->dtype == RN_BF16)
      hipLaunchKernelGGL(pack_krsc_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, wm,
                         (bf16_t*)w_krsc, d->k, RS, d->c_real, d->c);
    else
      hipLaunchKernelGGL(pack_krsc_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, wm,
                         (float*)w_krsc, d->k, RS, d->c_real, d->c);
  }
  if (w_crsk) {
    const int64_t total = (int64_t)d->c * RS * d->k_pad;
    if (d->dtype == RN_BF16)
      hipLaunchKernelGGL(pack_crsk_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, wm,
                         (bf16_t*)w_crsk, d->k, d->k_pad, RS, d->c_real, d->c);
    else
      hipLaunchKernelGGL(pack_crsk_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, wm,
                         (float*)w_crsk, d->k, d->k_pad, RS, d->c_real, d->c);
  }
  return rn_check_launch("weight_pack");
}

int rn_conv_weight_pack_multi(const rn_conv_desc* descs, const float* const* w_masters, void* const* w_krsc,
                              void* const* w_crsk, int32_t count, rn_stream_t stream) {
  RN_CHECK_ARG(count >= 0 && (count == 0 || (descs && w_masters && w_krsc && w_crsk)), "null argument");
  hipStream_t st = as_stream(stream);
  int32_t dtype = -1;
  for (int32_t i = 0; i < count; ++i) {
    const rn_conv_desc* d = descs + i;
    RN_CHECK_ARG(w_masters[i], "null master weight");
    if (d->groups <= 1) continue;
    RN_CHECK_ARG(d->c % d->groups == 0 && d->k % d->groups == 0, "channels not divisible by groups");
    RN_CHECK_ARG(dtype < 0 || dtype == d->dtype, "grouped copies of one call must share a dtype");
    dtype = d->dtype;
  }
  GpackBatch b;
  int nb = 0;
  int64_t most = 0;
  auto flush = [&]() {
    if (!nb) return;
    const dim3 grid((unsigned)std::min(grid_for(most), 1024), (unsigned)nb);
    if (dtype == RN_BF16)
      hipLaunchKernelGGL(pack_group_multi_kernel<bf16_t>, grid, dim3(256), 0, st, b);
    else
      hipLaunchKernelGGL(pack_group_multi_kernel<float>, grid, dim3(256), 0, st, b);
    nb = 0;
    most = 0;
  };
  for (int32_t i = 0; i < count; ++i) {
    const rn_conv_desc* d = descs + i;
    if (d->groups <= 1) {  // dense: the per-layer pack
      const int r = rn_conv_weight_pack(d, w_masters[i], w_krsc[i], w_crsk[i], stream);
      if (r) return r;
      continue;
    }
    const int cpg = d->c / d->groups, kpg = d->k / d->groups;
    for (int which = 0; which < 2; ++which) {
      void* out = which == 0 ? w_krsc[i] : w_crsk[i];
      if (!out) continue;
      GpackItem& p = b.it[nb];
      p.wm = w_masters[i];
      p.out = out;
      p.transpose = which;
      p.cpg = cpg;
      p.rs = d->r * d->s;
      p.direct = gd_direct_ok(d, which) ? 1 : 0;
      if (p.direct) {
        p.ncols = d->c;
        p.total = (int64_t)d->c * 9 * cpg;
        p.cblk = p.gcol = p.gred = 0;
      } else {
        p.ncols = which == 0 ? d->k : d->c;
        p.gcol = which == 0 ? kpg : cpg;
        p.gred = which == 0 ? cpg : kpg;
        p.cblk = group_blk(p.gcol, p.gred);
        p.total = (int64_t)p.ncols * p.rs * p.cblk;
      }
      most = std::max(most, p.total);
      if (++nb == kGpackMax) flush();
    }
  }
  flush();
  return rn_check_launch("weight_pack_multi");
}

}  // extern "C"

namespace {
int im2col_launch(const rn_conv_desc* d, const float* x, const float* scale, const float* shift, const float* qthr,
                  float qmax, void* cols, int32_t kc, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && cols, "null argument");
  RN_CHECK_ARG(kc >= d->r * d->s * d->c_real && kc % 8 == 0, "bad kc");
  RN_CHECK_ARG((scale == nullptr) == (shift == nullptr), "scale/shift must both be set");
  hipStream_t st = as_stream(stream);
  const FastDiv fq = make_fastdiv(d->q), fp = make_fastdiv(d->p), fc = make_fastdiv(d->c_real);
  if (d->dtype == RN_BF16) {
    const int64_t total = (int64_t)d->n * d->p * d->q * (kc / 8);
    hipLaunchKernelGGL(im2col_nchw_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, x,
                       scale, shift, (bf16_t*)cols, d->n, d->c_real, d->h, d->w, d->p, d->q, d->r,
                       d->s, d->stride_h, d->stride_w, d->pad_h, d->pad_w, kc, fq, fp, fc, qthr, qmax);
  } else {
    const int64_t total = (int64_t)d->n * d->p * d->q * (kc / 4);
    hipLaunchKernelGGL(im2col_nchw_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, x,
                       scale, shift, (float*)cols, d->n, d->c_real, d->h, d->w, d->p, d->q, d->r,
                       d->s, d->stride_h, d->stride_w, d->pad_h, d->pad_w, kc, fq, fp, fc, qthr, qmax);
  }
  return rn_check_launch("im2col");
}
}  // namespace

extern "C" {

int rn_im2col_nchw(const rn_conv_desc* d, const float* x, const float* scale, const float* shift,
                   void* cols, int32_t kc, rn_stream_t stream) {
  return im2col_launch(d, x, scale, shift, nullptr, 0.f, cols, kc, stream);
}

int rn_im2col_nchw_quant(const rn_conv_desc* d, const float* x, const float* scale, const float* shift,
                         float* minmax, int32_t is_train, float ema_decay, int32_t first_batch, int32_t nbits,
                         float* ws, void* cols, int32_t kc, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && minmax && ws, "null argument");
  RN_CHECK_ARG(nbits >= 2 && nbits <= 16, "bad nbits");
  hipStream_t st = as_stream(stream);
  float* curmax = ws;
  float* thr = ws + 1;
  hipMemsetAsync(curmax, 0, sizeof(float), st);
  if (is_train) {
    const int64_t total = (int64_t)d->n * d->c_real * d->h * d->w;
    hipLaunchKernelGGL(stem_affine_absmax_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, scale, shift, total,
                       d->c_real, d->h * d->w, curmax);
  }
  hipLaunchKernelGGL(stem_quant_state_kernel, dim3(1), dim3(1), 0, st, curmax, minmax, is_train, ema_decay,
                     first_batch, thr);
  if (rn_check_launch("im2col_quant_state")) return -1;
  return im2col_launch(d, x, scale, shift, thr, (float)((1 << (nbits - 1)) - 1), cols, kc, stream);
}

int rn_stem_quant_clip_grad(const rn_conv_desc* d, const float* x, const float* scale, const float* shift,
                            const float* minmax, const void* dy, const float* w_q, float* dbeta,
                            rn_stream_t stream) {
  RN_CHECK_ARG(d && x && minmax && dy && w_q && dbeta, "null argument");
  hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)d->n * d->c_real * d->h * d->w;
  RN_CHECK_ARG(total < (1ll << 31) - 64, "input exceeds 2^31 elements");
  RN_CHECK_ARG(d->c_real <= 8, "the quantized stem has at most 8 input channels");
  RN_CHECK_ARG(((uintptr_t)x & 15) == 0, "x must be 16-byte aligned");
  const size_t lds = (size_t)d->c_real * d->r * d->s * d->k * sizeof(float);  // the weights, [c][r][s][k]
  RN_CHECK_ARG(lds <= 64 * 1024, "stem weights exceed the LDS copy (c*r*s*k <= 16384)");
  RN_CHECK_ARG(d->k <= 64 && (d->r + d->stride_h - 1) / d->stride_h <= 4 && (d->s + d->stride_w - 1) / d->stride_w <= 4,
               "the quantized stem: k <= 64 and at most 4 x 4 taps per input pixel");
  RN_CHECK_ARG(d->k % 4 == 0 && d->k_pad % 4 == 0, "the quantized stem: k a multiple of 4");
  RN_CHECK_ARG(((uintptr_t)dy & 15) == 0, "dy must be 16-byte aligned");
  const ClipGeo gm{d->n, d->c_real, d->h, d->w, d->p, d->q, d->k, d->k_pad, d->r, d->s, d->stride_h, d->stride_w,
                   d->pad_h, d->pad_w, make_fastdiv(d->h * d->w), make_fastdiv(d->c_real), make_fastdiv(d->w),
                   make_fastdiv(d->stride_h), make_fastdiv(d->stride_w)};
  // blocks of 4 waves x 256 elements; at most ~8 per CU, each stages the weights once
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 1023) / 1024, 2048));
  if (d->dtype == RN_BF16)
    hipLaunchKernelGGL(stem_clip_grad_kernel<bf16_t>, dim3(blocks), dim3(256), lds, st, x, scale, shift,
                       minmax, (const bf16_t*)dy, w_q, dbeta, gm);
  else
    hipLaunchKernelGGL(stem_clip_grad_kernel<float>, dim3(blocks), dim3(256), lds, st, x, scale, shift,
                       minmax, (const float*)dy, w_q, dbeta, gm);
  return rn_check_launch("stem_quant_clip_grad");
}

int rn_stem_shift_grad(const rn_conv_desc* d, const void* dy, const float* wm, float* dbeta,
                       float* ws, rn_stream_t stream) {
  RN_CHECK_ARG(d && dy && wm && dbeta && ws, "null argument");
  hipStream_t st = as_stream(stream);
  const int PQ = d->p * d->q;
  const int64_t total = (int64_t)PQ * d->k_pad;
  RN_CHECK_ARG(d->k_pad % 8 == 0, "k_pad must be a multiple of 8");
  if (d->dtype == RN_BF16)
    hipLaunchKernelGGL(stem_sum_n_kernel<bf16_t>, dim3(grid_for(total / 8)), dim3(256), 0, st,
                       (const bf16_t*)dy, ws, d->n, PQ, d->k_pad);
  else
    hipLaunchKernelGGL(stem_sum_n_kernel<float>, dim3(grid_for(total / 4)), dim3(256), 0, st,
                       (const float*)dy, ws, d->n, PQ, d->k_pad);
  float* tq = ws + total;
  const int ntq = d->p * d->s * d->k;
  hipLaunchKernelGGL(stem_colsum_kernel, dim3((ntq + 255) / 256), dim3(256), 0, st, ws, tq, d->k, d->k_pad, d->s,
                     d->w, d->p, d->q, d->stride_w, d->pad_w);
  float* g = tq + ntq;
  const int nkt = d->k * d->r * d->s;
  hipLaunchKernelGGL(stem_tap_sum_kernel, dim3((nkt + 63) / 64), dim3(64), 0, st, tq, g, d->k, d->r, d->s, d->h,
                     d->p, d->stride_h, d->pad_h);
  hipLaunchKernelGGL(stem_shift_reduce_kernel, dim3(d->c_real), dim3(256), 0, st, g, wm, dbeta,
                     d->k, d->r * d->s, d->c_real);
  return rn_check_launch("stem_shift_grad");
}

}  // extern "C"

// ---- the int8 stem's clip gradient as a weight gradient (rn_stem_clip_mask / _wgrad / _dbeta)
// The input quantizer's straight-through clip removes from bn_data's beta gradient the data gradient
// at every clipped input: sum over clipped (n, c, h, w) of sum_{k,r,s} w[k,r,s,c] dy[n,p,q,k]. That is
// sum_{k,r,s} w[k,r,s,c] * D[k,r,s,c] with D the weight gradient of the stem convolution over the CLIP
// MASK of channel c: so the mask goes into the NHWC-8 image's free channels (c_real + c), the stem's
// weight gradient computes D with the real dW at no extra operand traffic (it reads all 8 channels
// anyway), and a 3-channel dot product finishes -- on the weight-gradient stream, instead of a gather
// of 16 dy rows per clipped input on the compute stream at the step's end (stem_clip_grad_kernel).
namespace {
__global__ __launch_bounds__(256) void stem_clip_mask_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ minmax, bf16_t* __restrict__ x8,
                                                             int64_t npix, int c, int hw) {
  const float t = *minmax;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i / hw, pix = i - img * hw;
    uint4 u = reinterpret_cast<const uint4*>(x8)[i];
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
    for (int e = 0; e < c; ++e) {
      const float v = fmaf(x[(img * c + e) * hw + pix], scale[e], shift[e]);
      const uint32_t m = (v > -t && v < t) ? 0u : 0x3F80u;  // bf16 1.0 where the clip zeroes the gradient
      const int ch = c + e;
      w[ch >> 1] = (ch & 1) ? ((w[ch >> 1] & 0x0000FFFFu) | (m << 16)) : ((w[ch >> 1] & 0xFFFF0000u) | m);
    }
    reinterpret_cast<uint4*>(x8)[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}
// dw[k][rs][c] += ext[k][rs][c] for c < c_real (ext: [k][rs][2 c_real], the real channels then the masks)
__global__ void stem_clip_split_kernel(const float* __restrict__ ext, float* __restrict__ dw, int krs, int c_real) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= krs * c_real) return;
  const int t = i / c_real, c = i - t * c_real;
  dw[i] += ext[(int64_t)t * 2 * c_real + c];
}
// dbeta[c] -= sum_{k,r,s} w[k][rs][c] * ext[k][rs][c_real + c]: one block per channel, a fixed order
__global__ __launch_bounds__(256) void stem_clip_dbeta_kernel(const float* __restrict__ ext, const float* __restrict__ w,
                                                              float* __restrict__ dbeta, int krs, int c_real) {
  const int c = blockIdx.x;
  float s = 0.f;
  for (int t = threadIdx.x; t < krs; t += blockDim.x) s = fmaf(w[(int64_t)t * c_real + c], ext[(int64_t)t * 2 * c_real + c_real + c], s);
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dbeta[c] -= red[0];
}
bool stem_clip_ok(const rn_conv_desc* d) {
  return d && d->dtype == RN_BF16 && d->groups <= 1 && d->c == 8 && d->c_real >= 1 && 2 * d->c_real <= 8;
}
rn_conv_desc stem_clip_ext(const rn_conv_desc* d) {  // the same convolution over the real + mask channels
  rn_conv_desc e = *d;
  e.c_real = 2 * d->c_real;
  return e;
}
}  // namespace

extern "C" {

int32_t rn_stem_clip_supported(const rn_conv_desc* d) { return stem_clip_ok(d) ? 1 : 0; }

int rn_stem_clip_mask(const rn_conv_desc* d, const float* x, const float* scale, const float* shift,
                      const float* minmax, void* x8, rn_stream_t stream) {
  RN_CHECK_ARG(d && x && scale && shift && minmax && x8, "null argument");
  RN_CHECK_ARG(stem_clip_ok(d), "the clip mask needs the bf16 NHWC-8 stem image with 2 * c_real <= 8");
  const int64_t npix = (int64_t)d->n * d->h * d->w;
  hipLaunchKernelGGL(stem_clip_mask_kernel, dim3(grid_for(npix)), dim3(256), 0, as_stream(stream), x, scale, shift,
                     minmax, (bf16_t*)x8, npix, d->c_real, d->h * d->w);
  return rn_check_launch("stem_clip_mask");
}

int64_t rn_stem_clip_wgrad_ws_bytes(const rn_conv_desc* d) {
  if (!stem_clip_ok(d)) return -1;
  const rn_conv_desc e = stem_clip_ext(d);
  return rn_conv_wgrad_ws_bytes(&e);
}

int rn_stem_clip_wgrad_chunk(const rn_conv_desc* d, const void* x8, const void* dy, float* dw, float* ext, void* ws,
                             int64_t ws_bytes, int32_t first, int32_t last, rn_stream_t stream) {
  RN_CHECK_ARG(d && x8 && dy && dw && ext, "null argument");
  RN_CHECK_ARG(stem_clip_ok(d), "the clip weight gradient needs the bf16 NHWC-8 stem image with 2 * c_real <= 8");
  const rn_conv_desc e = stem_clip_ext(d);
  const int krs = d->k * d->r * d->s;
  hipStream_t st = as_stream(stream);
  if (first && hipMemsetAsync(ext, 0, sizeof(float) * (size_t)krs * e.c_real, st) != hipSuccess)
    return rn_check_launch("stem_clip_wgrad");
  if (rn_conv_bwd_filter_ws(&e, x8, dy, ext, ws, ws_bytes, stream)) return -1;  // (adds into ext)
  if (!last) return 0;
  hipLaunchKernelGGL(stem_clip_split_kernel, dim3((krs * d->c_real + 255) / 256), dim3(256), 0, st, ext, dw, krs,
                     d->c_real);
  return rn_check_launch("stem_clip_wgrad");
}

int rn_stem_clip_wgrad(const rn_conv_desc* d, const void* x8, const void* dy, float* dw, float* ext, void* ws,
                       int64_t ws_bytes, rn_stream_t stream) {
  return rn_stem_clip_wgrad_chunk(d, x8, dy, dw, ext, ws, ws_bytes, 1, 1, stream);
}

int rn_stem_clip_dbeta(const rn_conv_desc* d, const float* ext, const float* w_q, float* dbeta, rn_stream_t stream) {
  RN_CHECK_ARG(d && ext && w_q && dbeta, "null argument");
  RN_CHECK_ARG(stem_clip_ok(d), "the clip gradient needs the bf16 NHWC-8 stem image with 2 * c_real <= 8");
  hipLaunchKernelGGL(stem_clip_dbeta_kernel, dim3(d->c_real), dim3(256), 0, as_stream(stream), ext, w_q, dbeta,
                     d->k * d->r * d->s, d->c_real);
  return rn_check_launch("stem_clip_dbeta");
}

}  // extern "C"
