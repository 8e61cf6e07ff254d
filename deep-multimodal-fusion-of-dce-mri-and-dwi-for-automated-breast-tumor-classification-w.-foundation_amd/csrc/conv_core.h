// Shared pieces of the gfx950 implicit-GEMM conv kernels (conv.hip, conv_pp.hip):
// launch arguments, activation helpers, the XCD-aware block remap, the BN
// statistics accumulator and the register epilogue of the 256x256 persistent
// tiles (operands swapped so each lane holds 16 output channels of one pixel).
#pragma once
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;


struct ConvArgs {
  const void* x;      // A source (FWD: input; DGRAD: dy)
  const void* w;      // B source [Nout][Ktot]
  const float* bias;  // [Nout] or null
  void* y;            // output NHWC, channel stride ldy
  float* partials;    // [mtiles][Nout][2] or null
  int N, H, W, C, ldx;  // A-source geometry (C = total channels over both sources)
  const void* x2;       // optional second source concatenated along channels (FWD only)
  int C1, ldx2;         // channels taken from x (the rest from x2), stride of x2
  int Ho, Wo, ldy;      // output geometry
  int Nout;             // GEMM N
  int KH, KW, stride, pad, dil;
  int Ktot;             // KH*KW*C
  int M;                // N*Ho*Wo
  int act;
  int act_in;
  int mtiles, ntiles;
  // A-operand prologue (FWD, single source): x <- act(x*in_ss[c] + in_ss[C+c])
  // on every in-bounds element (padding stays zero), i.e. the producer's
  // batch-norm apply + activation fused into this conv's loads.
  const float* in_ss;
  // fused batch-norm finalize: with `tickets` ([ntiles], zero at rest) the
  // last-arriving block of each output-channel tile reduces that tile's
  // columns of the partial-statistics slab (fixed order, double) and
  // finalizes them into `fin`, then re-zeroes its ticket.
  unsigned* tickets;
  BnFin fin;
  // stat_acc: the BN statistics are ADDED into (double*)partials [Nout][2]
  // (float64 atomics, zeroed by the caller) instead of one slab row per M
  // tile; the consumer (dmf_bn_apply) finalizes them
  int stat_acc;
  // benchmarking only (dmf_conv_tune key 6), k_conv_fwd_ps: bit 1 skips the
  // DMA (the loop then computes on stale LDS), bit 2 the epilogue, bit 3 its
  // stores, bit 4 its statistics; bit 5 makes the stores non-temporal (dmf_conv_tune key 6 only)
  int dbg;
  // affine epilogue of k_conv_fwd_ps (EPI 8 / 11, dmf_conv2d_fwd_affine): the BatchNorm already known,
  // y = relu(acc * out_ss[n] + out_ss[Nout + n] + r), r = res (EPI 8) or res * res_ss[n] + res_ss[Nout + n]
  // (EPI 11, the shortcut's own BatchNorm): conv -> BN -> + shortcut -> ReLU written once
  const float* out_ss;
  const void* res;
  int ldr;
  const float* res_ss;
  // aff_acc: EPI 8 / 11 take the BatchNorm's scale / shift from the float64 arena (partials, stat_acc
  // replicas, fin) when they stage them, instead of from out_ss (dmf_conv2d_fwd_affine_acc: the
  // finalize launch between the two passes folded in); block 0 also moves the running statistics
  int aff_acc;
  // residual epilogue of the conv_epilogue forms (buf / wide / sq / igemm; dmf_conv2d_fwd_res): after the
  // bias, y = act(y + res[m][n]) with res / ldr above -- an eval-mode Bottleneck conv3 whose BatchNorm is
  // folded into its weights and bias (dmf_ops._eval_fold)
  int res_add;
  // token-residual epilogue of k_conv_fwd_ps (EPI 15, dmf_conv2d_fwd_tokres): a transformer block's proj /
  // fc2 linear, out_f32 = res_f32 + colscale * dropout(acc + bias), the k_gemm_bf16 epilogue of those
  // linears (res / ldr: the f32 residual stream; y / ldy: f32 out; dp / rng / site: the dropout)
  int tok_res;
  const float* colscale;
  // dropout after the bias + GELU epilogue of k_conv_fwd_ps (EPI 14, dmf_conv2d_fwd_drop): Philox keep
  // masks on element m * Nout + n, the token GEMM's index (k_gemm_bf16 epilogue), so a forward-only
  // token block draws the same masks as the training path
  float dp;
  const unsigned long long* rng;
  int site;
  // in-kernel timing stamps (dmf_stamp_arm, tools/stream_stamps.py), null in production: this launch's
  // region of per-wave [start, end] s_memrealtime ticks (100 MHz, one clock for the whole chip)
  unsigned long long* stamp;
};

// Timing stamps without contention: lane 0 of every wave writes its own start / end (plain vector stores,
// no atomics -- one shared atomic per wave measurably stretched every launch) into this launch's region,
// [STAMP_MAX_BLOCKS blocks][8 waves][start, end]; the reader takes the min / max. One wave-uniform branch on
// the null pointer in production launches.
constexpr unsigned STAMP_MAX_BLOCKS = 4096;
struct StampScope {
  unsigned long long* q;
  __device__ __forceinline__ explicit StampScope(unsigned long long* p) : q(nullptr) {
    if (p) {
      const unsigned blk = blockIdx.x + blockIdx.y * gridDim.x, w = threadIdx.x >> 6;
      if (blk < STAMP_MAX_BLOCKS && w < 8 && (threadIdx.x & 63) == 0) {
        q = p + (blk * 8 + w) * 2;
        __builtin_nontemporal_store(wall_clock64(), q);
      }
    }
  }
  __device__ __forceinline__ ~StampScope() {
    if (q) __builtin_nontemporal_store(wall_clock64(), q + 1);
  }
};

template <int ACT>
__device__ __forceinline__ float apply_act(float v) {
  if (ACT == DMF_ACT_RELU) return fmaxf(v, 0.f);
  if (ACT == DMF_ACT_GELU) return gelu_f(v);
  if (ACT == DMF_ACT_SIGMOID) return sigmoid_f(v);
  return v;
}
__device__ __forceinline__ float apply_act_rt(int act, float v) {
  switch (act) {
    case DMF_ACT_RELU: return fmaxf(v, 0.f);
    case DMF_ACT_GELU: return gelu_f(v);
    case DMF_ACT_SIGMOID: return sigmoid_f(v);
    default: return v;
  }
}

// the activation over a whole register group with ONE uniform branch: a
// per-element apply_act_rt unrolls into a compare-and-branch chain per value
// and drags every activation's code through the instruction cache (the
// persistent conv's epilogue was ~40 % of its time that way)
template <int N>
__device__ __forceinline__ void apply_act_arr(int act, float (&v)[N]) {
  switch (act) {
    case DMF_ACT_RELU:
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = fmaxf(v[e], 0.f);
      break;
    case DMF_ACT_GELU:
      if constexpr (N % 2 == 0) {
#pragma unroll
        for (int e = 0; e < N; e += 2) {
          const dmf_f2 g = gelu_f2(dmf_f2{v[e], v[e + 1]});
          v[e] = g.x;
          v[e + 1] = g.y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < N; ++e) v[e] = gelu_f(v[e]);
      }
      break;
    case DMF_ACT_SIGMOID:
#pragma unroll
      for (int e = 0; e < N; ++e) v[e] = sigmoid_f(v[e]);
      break;
    default:
      break;
  }
}
template <int FM, int FN>
__device__ __forceinline__ void apply_act_col(int act, f32x4_t (&acc)[FM][FN], int j) {
  if (act == DMF_ACT_NONE) return;
  float v[FM * 4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[i * 4 + r] = acc[i][j][r];
  apply_act_arr(act, v);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[i][j][r] = v[i * 4 + r];
}

constexpr int CBM = 128, CBN = 128, CTHREADS = 256;
constexpr int STAGE_BYTES = (CBM + CBN) * 128;  // A + B, 128-byte rows
// main LDS: two A/B stages, reused for the C staging tile [BM][BN + 16 B pad]
__host__ __device__ constexpr int conv_lds_main(int esize, int bm = CBM, int bn = CBN) {
  return 2 * (bm + bn) * 128 > bm * (bn + 16 / esize) * esize ? 2 * (bm + bn) * 128 : bm * (bn + 16 / esize) * esize;
}
constexpr int CONV_LDS_EXTRA = 64 + CTHREADS * 2 * 8;  // flag + reducer doubles


constexpr int BUF_FLAGS_EP = 0x00020000;  // buffer descriptor word 3 (as BUF_FLAGS below)

// BN statistics of one column of one M tile into the accumulator (stat_acc):
// stat_acc = 1: float64 atomics into [Nout][2]; stat_acc = R > 1: into
// replica (mt % R) of [R][Nout][2] (spreads the same-address contention of
// the M tiles over R addresses; the consumer sums the replicas);
// stat_acc < 0: benchmarking variants (-1 f32 atomics, -2 plain slab store)
__device__ __forceinline__ void acc_stats(const ConvArgs& a, int mt, int col, float2 v) {
  if (a.stat_acc >= 1) {
    const int rep = a.stat_acc > 1 ? mt % a.stat_acc : 0;
    double* d = (double*)a.partials + ((size_t)rep * a.Nout + col) * 2;
    unsafeAtomicAdd(d, (double)v.x);
    unsafeAtomicAdd(d + 1, (double)v.y);
  } else if (a.stat_acc == -1) {
    unsafeAtomicAdd(a.partials + (size_t)col * 2, v.x);
    unsafeAtomicAdd(a.partials + (size_t)col * 2 + 1, v.y);
  } else {
    *(float2*)(a.partials + ((size_t)mt * a.Nout + col) * 2) = v;
  }
}

typedef unsigned v4u_t __attribute__((ext_vector_type(4)));

// (scale, shift) of channel c from the arena's replica sums in a fixed order -- the finalize k_bn_apply
// folds in (norm.hip bn_src_affine); `update`: this block also moves the running statistics (one block
// per channel: the tile row mt == 0). The replicas' (sum, sum^2) pairs are read with one 16-B sc1
// buffer load each (L1-bypassing), all eight in flight together. Used by the two-pass conv3's second
// pass (aff_acc: its BatchNorm finalized while it stages scale / shift).
constexpr int ARENA_MAX_REPLICAS = 8;
__device__ __forceinline__ float2 arena_bn_channel(const ConvArgs& a, int c, bool update) {
  const __amdgpu_buffer_rsrc_t rp =
      __builtin_amdgcn_make_buffer_rsrc(a.partials, 0, a.stat_acc * a.Nout * 16, BUF_FLAGS_EP);
  v4u_t pr[ARENA_MAX_REPLICAS];
#pragma unroll
  for (int r = 0; r < ARENA_MAX_REPLICAS; ++r)
    pr[r] = __builtin_bit_cast(v4u_t, __builtin_amdgcn_raw_buffer_load_b128(
                                          rp, r < a.stat_acc ? (unsigned)((r * a.Nout + c) * 16) : BUF_OOB, 0, 16));
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int r = 0; r < ARENA_MAX_REPLICAS; ++r) {
    s += __builtin_bit_cast(double, ((unsigned long long)pr[r].y << 32) | pr[r].x);
    q += __builtin_bit_cast(double, ((unsigned long long)pr[r].w << 32) | pr[r].z);
  }
  const BnFin& f = a.fin;
  const double m = s / f.count;
  double v = q / f.count - m * m;
  if (v < 0.0) v = 0.0;
  if (update && f.running_mean) {
    f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)m;
    const double n_ = f.unbias_count > 0.0 ? f.unbias_count : f.count;
    const double unb = n_ > 1.0 ? v * n_ / (n_ - 1.0) : v;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unb;
  }
  const float inv = rsqrtf((float)v + f.eps);
  const float g = f.gamma ? f.gamma[c] : 1.f, b = f.beta ? f.beta[c] : 0.f;
  return make_float2(g * inv, b - (float)m * g * inv);
}

constexpr int QBM = 256, QBN = 256, QSTAGE = (QBM + QBN) * 128;
constexpr int QWM = 2, QWN = 4, QTHREADS = 64 * QWM * QWN;
constexpr int QLDS_MAIN = 2 * QSTAGE > QBM * (QBN + 8) * 2 ? 2 * QSTAGE : QBM * (QBN + 8) * 2;
constexpr int QLDS = QLDS_MAIN + 64 + QTHREADS * 2 * 8;  // + epilogue flag and reducer doubles

constexpr int PS_LDS = 2 * QSTAGE + 2 * 256 * 2 * 4;  // ring + [2 halves][256 cols][2] stats (+ bias: Nout floats)

// local W-tile row -> channel offset within the 256-column tile: inside each
// 64-row wave slab, row 16j + 4g + r (bits j1 j0 g1 g0 r1 r0) holds channel
// 32*j1 + 8g + 4*j0 + r (bits j1 g1 g0 j0 r1 r0): a lane's accumulators of
// fragments j = 0,1 are channels 8g..8g+7, of j = 2,3 channels 32+8g..+7
__device__ __forceinline__ int ps_perm(int row) {
  const int slab = row & ~63, x = row & 63;
  return slab | (x & 0x23) | (((x >> 2) & 3) << 3) | (((x >> 4) & 1) << 2);
}
// channel offset (within the 256-column tile) of accumulator value e = 4j + r of lane group g in wave column wn
__device__ __forceinline__ int ps_chan(int wn, int g, int e) { return wn * 64 + g * 8 + (e & 7) + ((e >> 3) << 5); }

// Register epilogue of one 256x256 tile of the persistent forms (see
// k_conv_fwd_ps): bias (+ activation) or BN partial statistics, two 16-B
// buffer stores per pixel row straight from the accumulators. Every global
// access is issued unconditionally (out-of-range rows get BUF_OOB offsets) so
// a wave's vmem count is static: 16 stores (+2 float64 atomics in stat_acc
// mode, pixel-half wm == 0 only), all YOUNGER than the in-flight DMA, which
// the caller retires with a counted vmcnt.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
// reduce-scatter over the 16 lanes of a DPP row: returns the row's sum of
// v[lane & 15]. Four halving rounds (partners lane ^ 15 by row_mirror,
// (lane & 8) | (7 - lane & 7) by row_half_mirror, then quad xor 2 and xor 1):
// 15 exchanged values per lane instead of 64 shuffles of a full butterfly.
__device__ __forceinline__ float row_reduce_scatter16(float (&v)[16], int fr) {
  const bool b3 = fr & 8, b2 = fr & 4, b1 = fr & 2, b0 = fr & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float keep = b3 ? v[k + 8] : v[k], send = b3 ? v[k] : v[k + 8];
    v[k] = keep + dpp_f<0x140>(send);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float keep = b2 ? v[k + 4] : v[k], send = b2 ? v[k] : v[k + 4];
    v[k] = keep + dpp_f<0x141>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float keep = b1 ? v[k + 2] : v[k], send = b1 ? v[k] : v[k + 2];
    v[k] = keep + dpp_f<0x4E>(send);
  }
  const float keep = b0 ? v[1] : v[0], send = b0 ? v[0] : v[1];
  return keep + dpp_f<0xB1>(send);
}

// (FM pixel fragments per wave, TBM pixel rows per tile: 8 / 256 for the 256x256 forms, 4 / 128 for
// the 128x128 two-workgroup form; two pixel-half waves per channel slab in both)
template <int EPI, int TBN = QBN, int FM = 8, int TBM = QBM, typename T = bf16_t>
__device__ __forceinline__ void ps_epilogue(const ConvArgs& a, f32x4_t (&acc)[FM][4], int lin,
                                            __amdgpu_buffer_rsrc_t ry, float* sred, const float* sbias, int tid,
                                            int wm, int wn, int fr, int fg) {
  constexpr int FN = 4;
  const int mt = lin / a.ntiles, nt = lin - (lin / a.ntiles) * a.ntiles;
  const int m0 = mt * TBM, n0 = nt * TBN;
  const int cl = wn * 64 + fg * 8;  // this lane's channels: n0 + cl .. +7 and n0 + cl + 32 .. +39
  // EPI 0: BN statistics; EPI 5: the same for a launch without bias whose M is a multiple of the tile
  // height (every row in range: no bias adds, no row masks -- half the VALU of EPI 0);
  // EPI 8 / 11: affine (+ plain / BN'd residual) + ReLU with the statistics known (sbias holds them
  // staged, see below)
  // EPI 12: EPI 5's statistics only, no output stores (the first pass of a conv whose BatchNorm is then
  // applied by the second, affine pass -- dmf_conv2d_fwd_stats)
  constexpr bool stats = EPI == 0 || EPI == 5 || EPI == 12, fast = EPI == 5 || EPI == 12, nostore = EPI == 12;
  constexpr bool aff = EPI == 8 || EPI == 11, rbn = EPI == 11;
  // EPI 14: the Philox (seed, offset) once per tile
  unsigned long long dseed = 0, doff = 0;
  float dks = 1.f;
  if constexpr (EPI == 14) {
    dseed = a.rng[0];
    doff = a.rng[1];
    dks = 1.f / (1.f - a.dp);
  }
  // staged [scale | shift (+ the residual's shift) | residual scale] x Nout (k_conv_fwd_ps)
  float bsv[16], shv[16], rsv[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int n = n0 + ps_chan(wn, fg, e);
    bsv[e] = aff ? sbias[n] : ((!fast && a.bias) ? sbias[n] : 0.f);
    shv[e] = aff ? sbias[a.Nout + n] : 0.f;
    rsv[e] = rbn ? sbias[2 * a.Nout + n] : 1.f;
  }
  const __amdgpu_buffer_rsrc_t rres =
      __builtin_amdgcn_make_buffer_rsrc(aff ? const_cast<void*>(a.res) : a.y, 0,
                                        (int)((long long)a.M * (aff ? a.ldr : a.ldy) * (int)sizeof(T)), BUF_FLAGS_EP);
  // affine epilogue: every fragment's shortcut loads in flight together (one exposed latency per tile)
  v4u_t rsd[aff ? FM : 1][2];
  if constexpr (aff) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * (TBM / 2) + i * 16 + fr;
      const bool ok = m < a.M;
      const unsigned ro = ok ? (unsigned)(((size_t)m * a.ldr + n0 + cl) * sizeof(T)) : BUF_OOB;
      rsd[i][0] = __builtin_bit_cast(v4u_t, __builtin_amdgcn_raw_buffer_load_b128(rres, ro, 0, 0));
      rsd[i][1] = __builtin_bit_cast(v4u_t, __builtin_amdgcn_raw_buffer_load_b128(rres, ok ? ro + 64 : BUF_OOB, 0, 0));
    }
  }
  float s[16], q[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) { s[e] = 0.f; q[e] = 0.f; }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * (TBM / 2) + i * 16 + fr;
    const bool ok = fast || m < a.M;
    float v[16];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[j * 4 + r] = fast ? acc[i][j][r] : (aff ? __builtin_fmaf(acc[i][j][r], bsv[j * 4 + r], shv[j * 4 + r])
                                                  : acc[i][j][r] + bsv[j * 4 + r]);
    if constexpr (aff) {
      // the shortcut: 16 channels of pixel m (two 16-B loads issued for every fragment up front),
      // plain or through its own BatchNorm
      const v4u_t r0 = rsd[i][0], r1 = rsd[i][1];
      const uint32_t rw[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float lo = B16<T>::lo(rw[k]), hi = B16<T>::hi(rw[k]);
        v[2 * k] = fmaxf(rbn ? __builtin_fmaf(lo, rsv[2 * k], v[2 * k]) : v[2 * k] + lo, 0.f);
        v[2 * k + 1] = fmaxf(rbn ? __builtin_fmaf(hi, rsv[2 * k + 1], v[2 * k + 1]) : v[2 * k + 1] + hi, 0.f);
      }
    }
    if (fast) {
#pragma unroll
      for (int e = 0; e < 16; ++e) { s[e] += v[e]; q[e] = __builtin_fmaf(v[e], v[e], q[e]); }
    } else if (stats) {
      const float w = ok ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) { s[e] += w * v[e]; q[e] += w * v[e] * v[e]; }
    } else if constexpr (EPI - 1 == DMF_ACT_GELU || EPI == 14) {
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const dmf_f2 g = gelu_f2(dmf_f2{v[e], v[e + 1]});
        v[e] = g.x;
        v[e + 1] = g.y;
      }
      if constexpr (EPI == 14) {
        // values 8h .. 8h+7 are channels n0 + cl + 32 h .. +7 of row m
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int q4 = 0; q4 < 2; ++q4) {
            bool keep[4];
            dropout_keep4v(dseed, doff, a.site, (unsigned long long)m * a.Nout + n0 + cl + 32 * h + 4 * q4, a.dp, keep);
#pragma unroll
            for (int t = 0; t < 4; ++t) v[8 * h + 4 * q4 + t] = keep[t] ? v[8 * h + 4 * q4 + t] * dks : 0.f;
          }
      }
    } else if constexpr (EPI > 1 && EPI < 5) {
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = apply_act<(EPI < 5 ? EPI - 1 : 0)>(v[e]);
    }
    uint32_t w8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) w8[e] = B16<T>::pack(v[2 * e], v[2 * e + 1]);
    const unsigned off = ok ? (unsigned)(((size_t)m * a.ldy + n0 + cl) * 2) : BUF_OOB;
    if (nostore) {
    } else if (a.dbg & 32) {
      __builtin_amdgcn_raw_buffer_store_b128(v4u_t{w8[0], w8[1], w8[2], w8[3]}, ry, off, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(v4u_t{w8[4], w8[5], w8[6], w8[7]}, ry, ok ? off + 64 : BUF_OOB, 0, 2);
    } else if (!(a.dbg & 8)) {
      __builtin_amdgcn_raw_buffer_store_b128(v4u_t{w8[0], w8[1], w8[2], w8[3]}, ry, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(v4u_t{w8[4], w8[5], w8[6], w8[7]}, ry, ok ? off + 64 : BUF_OOB, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  if (stats && !(a.dbg & 16)) {
    // lane fr of lane group fg ends with the 16 pixel lanes' totals of value fr's channel
    const float S = row_reduce_scatter16(s, fr), Q = row_reduce_scatter16(q, fr);
    const int ch = ps_chan(wn, fg, fr);
    if (a.stat_acc) {
      // the two pixel-half waves of each channel slab meet in LDS: half the atomics
      // (the K-step barriers order this slot's reuse by the next tile's epilogue)
      if (wm == 1) {
        sred[ch * 2] = S;
        sred[ch * 2 + 1] = Q;
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (wm == 0) acc_stats(a, mt, n0 + ch, make_float2(S + sred[ch * 2], Q + sred[ch * 2 + 1]));
    } else {
      // combine the two pixel-half waves through LDS, then one slab row per M tile
      sred[(wm * TBN + ch) * 2] = S;
      sred[(wm * TBN + ch) * 2 + 1] = Q;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid < TBN) {
        const float2 v = make_float2(sred[tid * 2] + sred[(TBN + tid) * 2],
                                     sred[tid * 2 + 1] + sred[(TBN + tid) * 2 + 1]);
        *(float2*)(a.partials + ((size_t)mt * a.Nout + n0 + tid) * 2) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
}

// Register epilogue of EPI 15 (see ConvArgs::tok_res) for the 256x256 persistent form: the lane's 16
// channels of each pixel row (ps_chan) get + bias, the token GEMM's Philox keep mask on element
// m * Nout + n (the same masks as k_gemm_bf16's epilogue), x colscale, + the f32 residual, and leave as
// four 16-B f32 stores. Kept light on registers (it is inlined into the K loop's body): bias / colscale
// re-read from LDS per fragment row, the residual loaded one fragment row ahead (2 x 4 loads in flight).
template <int TBN = QBN, int FM = 8, int TBM = QBM>
__device__ __forceinline__ void ps_epilogue_tokres(const ConvArgs& a, f32x4_t (&acc)[FM][4], int lin,
                                                   const float* sbias, int wm, int wn, int fr, int fg) {
  const int mt = lin / a.ntiles, nt = lin - (lin / a.ntiles) * a.ntiles;
  const int m0 = mt * TBM, n0 = nt * TBN;
  const int cl = wn * 64 + fg * 8;
  const bool drop = a.dp > 0.f;
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.res), 0, (int)((long long)a.M * a.ldr * 4), BUF_FLAGS_EP);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)((long long)a.M * a.ldy * 4), BUF_FLAGS_EP);
  // chunk q of a row: channels cl + 4 (q & 1) + 32 (q >> 1) .. +3 = values 4q .. 4q+3 (ps_chan)
  auto load_res = [&](int i, v4u_t (&rv)[4]) {
    const int m = m0 + wm * (TBM / 2) + i * 16 + fr;
    const unsigned ro = (unsigned)(((size_t)m * a.ldr + n0 + cl) * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      rv[q] = __builtin_bit_cast(v4u_t, __builtin_amdgcn_raw_buffer_load_b128(
                                            rr, m < a.M ? ro + (q & 1) * 16 + (q >> 1) * 128 : BUF_OOB, 0, 0));
  };
  v4u_t rcur[4], rnext[4];
  load_res(0, rcur);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if (i + 1 < FM) load_res(i + 1, rnext);
    const int m = m0 + wm * (TBM / 2) + i * 16 + fr;
    float v[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + cl + (q & 1) * 4 + (q >> 1) * 32;
      const float4 bq = *(const float4*)(sbias + n);
      const float bb[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) v[4 * q + t] = acc[i][q][t] + bb[t];
    }
    if (drop) {
      const float dks = 1.f / (1.f - a.dp);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bool keep[4];
        dropout_keep4v(a.rng[0], a.rng[1], a.site,
                       (unsigned long long)m * a.Nout + n0 + cl + (q & 1) * 4 + (q >> 1) * 32, a.dp, keep);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[4 * q + t] = keep[t] ? v[4 * q + t] * dks : 0.f;
      }
    }
    const unsigned yo = (unsigned)(((size_t)m * a.ldy + n0 + cl) * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + cl + (q & 1) * 4 + (q >> 1) * 32;
      const float4 g = *(const float4*)(sbias + a.Nout + n);
      const v4u_t r = rcur[q];
      v4u_t o;
      o.x = __float_as_uint(__builtin_fmaf(v[4 * q], g.x, __uint_as_float(r.x)));
      o.y = __float_as_uint(__builtin_fmaf(v[4 * q + 1], g.y, __uint_as_float(r.y)));
      o.z = __float_as_uint(__builtin_fmaf(v[4 * q + 2], g.z, __uint_as_float(r.z)));
      o.w = __float_as_uint(__builtin_fmaf(v[4 * q + 3], g.w, __uint_as_float(r.w)));
      __builtin_amdgcn_raw_buffer_store_b128(o, ry, m < a.M ? yo + (q & 1) * 16 + (q >> 1) * 128 : BUF_OOB, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) rcur[q] = rnext[q];
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (the instruction takes an immediate): one
// scalar branch per call
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
#define DMF_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    DMF_VMW(0) DMF_VMW(1) DMF_VMW(2) DMF_VMW(3) DMF_VMW(4) DMF_VMW(5) DMF_VMW(6) DMF_VMW(7)
    DMF_VMW(8) DMF_VMW(9) DMF_VMW(10) DMF_VMW(11) DMF_VMW(12) DMF_VMW(13) DMF_VMW(14) DMF_VMW(15)
    DMF_VMW(16) DMF_VMW(17) DMF_VMW(18) DMF_VMW(19) DMF_VMW(20) DMF_VMW(21) DMF_VMW(22) DMF_VMW(23)
    DMF_VMW(24) DMF_VMW(25) DMF_VMW(26) DMF_VMW(27) DMF_VMW(28) DMF_VMW(29) DMF_VMW(30) DMF_VMW(31)
    DMF_VMW(32) DMF_VMW(33) DMF_VMW(34) DMF_VMW(35) DMF_VMW(36) DMF_VMW(37) DMF_VMW(38) DMF_VMW(39)
    DMF_VMW(40) DMF_VMW(41) DMF_VMW(42) DMF_VMW(43) DMF_VMW(44) DMF_VMW(45) DMF_VMW(46) DMF_VMW(47)
    DMF_VMW(48) DMF_VMW(49) DMF_VMW(50) DMF_VMW(51) DMF_VMW(52) DMF_VMW(53) DMF_VMW(54) DMF_VMW(55)
    DMF_VMW(56) DMF_VMW(57) DMF_VMW(58) DMF_VMW(59) DMF_VMW(60) DMF_VMW(61) DMF_VMW(62)
#undef DMF_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// 7x7 / stride-2 stem conv (conv_stem.hip): legality, pixels per workgroup (= BN slab rows), launcher
bool conv_stem_ok(int dtype, bool dgrad, const ConvArgs& a);
int conv_stem_m_tile(const ConvArgs& a);
int launch_conv_stem(ConvArgs& a, hipStream_t st, int dtype);

// persistent / ping-pong 256x256 launcher of conv_pp.hip (epi: 0 / 5 BN statistics, 1 + act: bias + act)
int launch_conv_pp(ConvArgs& a, int epi, bool plain, size_t lds_bias, hipStream_t st, int dtype);
int conv_pp_tune(int value);  // dmf_conv_tune key 8
constexpr int PP_THREADS = 512;
constexpr int PP_HALF = 128 * 128;  // one half-tile: 128 rows x 128 B
constexpr int PP_SLOT = 4 * PP_HALF;  // a K-tile: pixel halves P0 P1, channel halves C0 C1
constexpr int PP_LDS = 2 * PP_SLOT + 2 * 256 * 2 * 4;  // two K-tile slots + epilogue statistics scratch (+ bias)

}  // namespace dmf
