// The ResNet-50 stem: 7x7 / stride 2 / pad 3 convolution, 64 output channels,
// over NHWC bf16 input with 8 or 16 (zero-padded) channels (timm's conv1,
// reference foundation_model.py:260-267 via build_medical_backbone; the DWI
// stem takes 14 -> 16 channels, the DCE stem 6 -> 8, config 2's 5 -> 8).
//
// The general implicit GEMM runs this shape at ~0.11 of its roofline: K =
// 49 * C is not a multiple of its 64-channel K-step, so every K-step gathers
// through the slow path. Here the K axis is ordered the way the input lies
// in memory: one 32-wide MFMA K-chunk is CP = 32 / C horizontally adjacent
// taps of one filter row x all C channels -- 64 contiguous bytes of one input
// row (taps past the 7th carry zero weights: 7 * ceil(7 / CP) chunks, 28 for
// C = 16, 14 for C = 8).
//
// Workgroup = 4 waves, one per SIMD; wave w owns output channels 16w..16w+15
// and keeps their weights for every K-chunk in VGPRs for the whole kernel
// (the MFMA row operand). A workgroup walks `rpw` consecutive output rows of
// one image; the 7 input rows an output row needs sit in a 9-row LDS ring
// (stride 2: each step brings in 2 new rows, staged by LDS-DMA one step
// ahead, the zero padding from the buffer range check). The column operand is
// read straight from the ring: a 16x32 pixel fragment is 1 KiB of one row.
// For C = 16 a row keeps its two 8-channel halves in two planes whose bases
// differ by an odd number of 16-B slots, which makes those reads free of LDS
// bank conflicts under gfx950's ds_read_b128 lane grouping (C = 8 is
// conflict-free as is).
//
// Epilogue (per 64-pixel column block): optional bias (+ activation without
// statistics: eval-mode BatchNorm folded into the weights), bf16 stores, 4
// channels x 8 B per lane; in the training forward the BN batch statistics of the workgroup's
// pixels are summed in registers across all its rows and added once at the end
// (float64 arena replicas, or one slab row per workgroup).
#include <algorithm>
#include <type_traits>

#include "conv_core.h"

namespace dmf {

constexpr int STEM_SLOTS = 9;  // 7 rows in use + the next step's 2

// C: padded input channels (8 / 16); STATS: BN statistics epilogue (a.partials)
template <int C, bool STATS, bool F16 = false>
__global__ void __launch_bounds__(256) k_conv_stem(ConvArgs a, int rpw, int plane) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  typedef typename std::conditional<F16, f16_t, bf16_t>::type T;  // storage type (bf16 / f16)
  constexpr int NPL = C / 8;               // 16-B channel planes per pixel
  constexpr int CP = 32 / C;               // taps per K-chunk
  constexpr int TG = (7 + CP - 1) / CP;    // K-chunks per filter row
  constexpr int NCH = 7 * TG;              // K-chunks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int pl1 = NPL == 2 ? plane + 16 : 0;      // odd number of 16-B slots past plane 0
  const int slot = NPL == 2 ? 2 * plane + 16 : plane;
  const int npp = plane / 1024;                   // DMA pieces per plane
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const int wg_per_img = a.Ho / rpw;
  const int n = blockIdx.x / wg_per_img;
  const int ho0 = (blockIdx.x - n * wg_per_img) * rpw, ho1 = ho0 + rpw;

  // this wave's 16 output channels: weights of every K-chunk (row operand), loaded before any DMA
  // is issued ([Cout][7][7][C] bf16; taps past the 7th are zero)
  const int co = wid * 16 + fr;
  uint4 wf[NCH];
  {
    const char* W = (const char*)a.w;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int r = c / TG, g = c % TG;
      const int s = g * CP + (fg * 8) / C, ci = (fg * 8) % C;
      wf[c] = s < 7 ? *(const uint4*)(W + ((size_t)((co * 7 + r) * 7 + s) * C + ci) * 2) : make_uint4(0, 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const v4i_t rx = buf_rsrc(a.x, (long long)a.N * a.H * a.W * C * 2);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)((long long)a.M * a.ldy * 2), BUF_FLAGS);

  // stage input row hi (zero rows / columns outside the image) into its ring slot: piece j of the
  // row is issued by wave j % 4
  auto stage_row = [&](int hi) {
    const unsigned base = lds0 + (unsigned)((hi + 3) % STEM_SLOTS) * slot;
    const bool rok = (unsigned)hi < (unsigned)a.H;
    for (int j = wid; j < NPL * npp; j += 4) {
      const int pl = j / npp, k = j - (j / npp) * npp;
      const int p = (k * 1024 + lane * 16) / 16;  // padded pixel index of this lane's 16 B
      const int wi = p - 3;
      const bool ok = rok && (unsigned)wi < (unsigned)a.W;
      const unsigned vo = ok ? (unsigned)((((size_t)(n * a.H + hi) * a.W + wi) * C + pl * 8) * 2) : BUF_OOB;
      dma16(rx, vo, 0, base + pl * pl1 + k * 1024);
    }
  };

  for (int k = 0; k < 7; ++k) stage_row(2 * ho0 - 3 + k);
  float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  // bias (an eval-mode BatchNorm folded into the weights: dmf_ops._eval_fold) of this lane's 4 channels
  float bj[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = a.bias[wid * 16 + fg * 4 + j];
  }
  const int ncb = a.Wo / 64;  // 64-pixel column blocks per output row
  int prev_st = 0;            // stores the previous step issued (younger than the rows this step needs)
  for (int ho = ho0; ho < ho1; ++ho) {
    vm_wait_rt(prev_st);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // the next step's two new rows go into the slots of rows 2ho-5, 2ho-4 (read last by step ho-1)
    if (ho + 1 < ho1) {
      stage_row(2 * ho + 4);
      stage_row(2 * ho + 5);
    }
    unsigned rb[7];
#pragma unroll
    for (int r = 0; r < 7; ++r) rb[r] = (unsigned)((2 * ho + r) % STEM_SLOTS) * slot;
    for (int cb = 0; cb < ncb; ++cb) {
      f32x4_t acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int r = c / TG, g = c % TG;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int wo = cb * 64 + i * 16 + fr;
          const int p = C == 16 ? 2 * wo + 2 * g + (fg >> 1) : 2 * wo + 4 * g + fg;
          const int pl = C == 16 ? (fg & 1) : 0;
          const uint4 pv = *(const uint4*)(smem + rb[r] + pl * pl1 + p * 16);
          acc[i] = mfma16<T>(wf[c], pv, acc[i]);
        }
      }
      // lane: pixel wo = cb*64 + 16i + fr, channels 16 wid + 4 fg + 0..3
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = (n * a.Ho + ho) * a.Wo + cb * 64 + i * 16 + fr;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[i][j] + bj[j];
        if (!STATS) apply_act_arr(a.act, v);  // (the statistics path runs act-free: the BN apply follows)
        uint32_t w2[2];
        w2[0] = B16<T>::pack(v[0], v[1]);
        w2[1] = B16<T>::pack(v[2], v[3]);
        const unsigned off = (unsigned)(((size_t)m * a.ldy + wid * 16 + fg * 4) * 2);
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, w2), ry, off, 0, 0);
        if (STATS) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s[j] += v[j];
            q[j] = __builtin_fmaf(v[j], v[j], q[j]);
          }
        }
      }
    }
    prev_st = 4 * ncb;
  }
  if (STATS) {
    // the 16 pixel lanes of each channel group
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s[j] += __shfl_xor(s[j], o, 64);
        q[j] += __shfl_xor(q[j], o, 64);
      }
    }
    if (fr == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc_stats(a, blockIdx.x, wid * 16 + fg * 4 + j, make_float2(s[j], q[j]));
    }
  }
}

// output rows per workgroup (one image per workgroup): the largest divisor of Ho that is <= 16 and
// still gives >= 256 workgroups (one per CU), else the smallest that does
static int stem_rows(int N, int Ho) {
  int best = 1;
  for (int r = 1; r <= 16; ++r)
    if (Ho % r == 0 && (long long)N * (Ho / r) >= 256) best = r;
  return best;
}

static int stem_plane(int W) { return (((W + 6) * 16 + 1023) / 1024) * 1024; }

bool conv_stem_ok(int dtype, bool dgrad, const ConvArgs& a) {
  if (!is16(dtype) || dgrad || a.KH != 7 || a.KW != 7 || a.stride != 2 || a.pad != 3 || a.dil != 1) return false;
  if ((a.C != 8 && a.C != 16) || a.ldx != a.C || a.x2 != nullptr || a.in_ss != nullptr || a.tickets != nullptr)
    return false;
  // bias in either mode; an activation only without the statistics epilogue (whose callers pass none)
  if (a.Nout != 64 || (a.act != DMF_ACT_NONE && a.partials != nullptr) || a.ldy % 4 != 0) return false;
  if (a.Wo % 64 != 0 || a.W != 2 * a.Wo || a.H != 2 * a.Ho) return false;
  const int plane = stem_plane(a.W);
  const long long lds = (long long)STEM_SLOTS * (a.C == 16 ? 2 * plane + 16 : plane);
  if (lds > 160 * 1024) return false;
  return (long long)a.M * a.ldy * 2 < (1LL << 31) && (long long)a.N * a.H * a.W * a.C * 2 < (1LL << 31);
}

// pixels per workgroup (the BN statistics slab has one row per workgroup)
int conv_stem_m_tile(const ConvArgs& a) { return stem_rows(a.N, a.Ho) * a.Wo; }

int launch_conv_stem(ConvArgs& a, hipStream_t st, int dtype) {
  const int rpw = stem_rows(a.N, a.Ho);
  const int plane = stem_plane(a.W);
  const size_t lds = (size_t)STEM_SLOTS * (a.C == 16 ? 2 * plane + 16 : plane);
  const dim3 g((unsigned)(a.N * (a.Ho / rpw))), b(256);
  const bool stats = a.partials != nullptr;
#define DMF_STEM(F)                                                                      \
  do {                                                                                   \
    if (a.C == 16) {                                                                     \
      if (stats) hipLaunchKernelGGL((k_conv_stem<16, true, F>), g, b, lds, st, a, rpw, plane);  \
      else hipLaunchKernelGGL((k_conv_stem<16, false, F>), g, b, lds, st, a, rpw, plane);       \
    } else {                                                                             \
      if (stats) hipLaunchKernelGGL((k_conv_stem<8, true, F>), g, b, lds, st, a, rpw, plane);   \
      else hipLaunchKernelGGL((k_conv_stem<8, false, F>), g, b, lds, st, a, rpw, plane);        \
    }                                                                                    \
  } while (0)
  if (dtype == DMF_F16) DMF_STEM(true);
  else DMF_STEM(false);
#undef DMF_STEM
  DMF_LAUNCH_CHECK("conv_stem");
  return 0;
}

}  // namespace dmf
