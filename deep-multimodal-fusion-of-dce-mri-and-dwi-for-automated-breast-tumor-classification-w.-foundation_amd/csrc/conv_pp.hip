// Implicit-GEMM forward conv, 256x256 tile, "ping-pong" K loop (gfx950).
//
// Same GEMM view, operand roles and register epilogue as k_conv_fwd_ps
// (conv.hip): pixels are the MFMA column operand, weights the row operand
// with the rows of each wave's 64-channel slab loaded in the ps_perm order,
// so after the K loop a lane holds 16 output channels of each of its pixels
// and ps_epilogue stores / reduces them straight from the accumulators.
//
// What changes is the K loop. 8 waves (2 pixel halves x 4 channel quarters,
// 128x64 outputs each, two waves per SIMD). A K-tile (BK = 64) is split into
// four HALF-tiles of 16 KiB each -- pixel halves P0 / P1 (the 64-pixel
// halves of every wave's 128 pixels) and channel halves C0 / C1 (the 32-
// channel halves of every wave's 64) -- and computed in four PHASES, one
// output quadrant (64 pixels x 32 channels x K 64 = 16 MFMAs) each:
//   phase 0 (P0,C0): read P0 + C0 fragments   stage C1 of K-tile t+1
//   phase 1 (P0,C1): read C1                   stage P1 of K-tile t+1
//   phase 2 (P1,C1): read P1                   stage P0 of K-tile t+2
//   phase 3 (P1,C0): (C0 kept)                 stage C0 of K-tile t+2
// A phase is two barrier intervals: a LOAD segment (its fragment reads, its
// two LDS-DMA pieces, a counted vmcnt) and an MFMA segment (16 MFMAs at
// s_setprio 1). Waves 4-7 start one barrier later than waves 0-3, so on every
// SIMD one wave computes while its partner loads (MI355X_MICROARCH.md "Two
// waves per SIMD"; cdna_hip_programming.md "The 256^2 8-phase template").
// Half-tiles are issued in exactly the order they are consumed, two K-tile
// slots of LDS (128 KiB), four half-tiles in flight: each phase's wait
// retires the half its NEXT phase reads (read one phase after the wait),
// and a half is restaged >= 2 phases after its last read.
#include <algorithm>
#include <type_traits>

#include "conv_core.h"

namespace dmf {

// row of the weight tile (0..255) that LDS row rho of channel half ch holds:
// wave slab rho >> 5, slab row 32*ch + (rho & 31) in the ps_perm order
__device__ __forceinline__ int pp_chan_row(int ch, int rho) {
  return ps_perm(((rho >> 5) << 6) | (ch << 5) | (rho & 31));
}
// tile pixel that LDS row rho of pixel half ph holds: wave half rho >> 6, pixel 64*ph + (rho & 63) of it
__device__ __forceinline__ int pp_pix_row(int ph, int rho) { return ((rho >> 6) << 7) | (ph << 6) | (rho & 63); }

// dma16 with its scalar operands forced into SGPRs (under this kernel's register pressure hipcc may keep
// a wave-uniform descriptor in VGPRs, which the inline asm's "s" operands cannot take)
__device__ __forceinline__ void dma16u(v4i_t rsrc, unsigned voff, unsigned soff, unsigned lds) {
  const v4i_t r = v4i_t{__builtin_amdgcn_readfirstlane(rsrc[0]), __builtin_amdgcn_readfirstlane(rsrc[1]),
                        __builtin_amdgcn_readfirstlane(rsrc[2]), __builtin_amdgcn_readfirstlane(rsrc[3])};
  dma16(r, voff, (unsigned)__builtin_amdgcn_readfirstlane((int)soff), (unsigned)__builtin_amdgcn_readfirstlane((int)lds));
}

// s_barrier that is also a compiler memory barrier: the builtin is not one, so hipcc may hoist the next
// phase's LDS fragment reads above it -- ahead of the partner group's DMA wait (a race)
__device__ __forceinline__ void pp_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PERSISTENT grid: gridDim <= tiles, each block walks tiles blockIdx, +gridDim, ... (XCD remap) as ONE
// flat stream of K-tiles: the staging runs two K-tiles ahead across tile boundaries, so the next
// tile's first half-tiles are in flight under the finished tile's epilogue (its 16 stores, +2 float64
// atomics in statistics mode, are then younger than those DMA pieces: the first K-tile after an
// epilogue waits with 16 more).
template <bool PADCHK, bool DUAL, int EPI, typename T = bf16_t>
__global__ void __launch_bounds__(PP_THREADS, 1) k_conv_fwd_pp(ConvArgs a) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  constexpr int ES = 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;  // source-side swizzle: LDS chunk (lane & 7) of row lr holds logical chunk lc
  const int fr = lane & 15, fg = lane >> 4;
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  float* sred = (float*)(smem + 2 * PP_SLOT);
  float* sbias = sred + 2 * 256 * 2;
  const int ntile = a.mtiles * a.ntiles;
  if ((int)blockIdx.x >= ntile) return;
  if (a.bias) {
    for (int i = tid; i < a.Nout; i += PP_THREADS) sbias[i] = a.bias[i];
    __syncthreads();
  }

  const v4i_t rx = buf_rsrc(a.x, (long long)a.N * a.H * a.W * a.ldx * ES);
  const v4i_t rx2 = buf_rsrc(DUAL ? a.x2 : a.x, (long long)a.N * a.H * a.W * (DUAL ? a.ldx2 : a.ldx) * ES);
  const v4i_t rw = buf_rsrc(a.w, (long long)a.Nout * a.Ktot * ES);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)((long long)a.M * a.ldy * ES), BUF_FLAGS);
  const int nk = a.Ktot / 64;
  const int hw = a.Ho * a.Wo;
  const int G = ((ntile - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x) * nk;  // this block's K-tiles
  auto tile_lin = [&](int j) { return xcd_remap((int)blockIdx.x + j * (int)gridDim.x, ntile); };

  // staging rows of the tile being STAGED: piece q (0, 1) of a half covers half rows 16*wid + 8*q + (0..7)
  int h0[2][2], w0[2][2], b1[2][2], b2[2][2];
  bool mok[2][2];
  unsigned vb[2][2];
  int meta_tile = -1;
  auto rows_for = [&](int j) {
    const int lin = tile_lin(j);
    const int mt = lin / a.ntiles, nt = lin - (lin / a.ntiles) * a.ntiles;
    const int m0 = mt * 256, n0 = nt * 256;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rho = 16 * wid + 8 * q + lr;
        const int m = m0 + pp_pix_row(ph, rho);
        mok[ph][q] = m < a.M;
        const int mm = mok[ph][q] ? m : 0;
        const int n = mm / hw, rem = mm - (mm / hw) * hw;
        const int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
        h0[ph][q] = ho * a.stride - a.pad;
        w0[ph][q] = wo * a.stride - a.pad;
        const int pix = (n * a.H + h0[ph][q]) * a.W + w0[ph][q];
        b1[ph][q] = pix * a.ldx + lc * 8;
        b2[ph][q] = DUAL ? pix * a.ldx2 + lc * 8 : 0;
        const int co = n0 + pp_chan_row(ph, rho);  // (ph doubles as the channel half index here)
        vb[ph][q] = (unsigned)((co * a.Ktot + lc * 8) * ES);
      }
    meta_tile = j;
  };

  // K-tile parameters (wave-uniform) from a division-free cursor over the flat stream: channel chunk
  // outer, filter tap inner (the taps of one chunk re-read L2-resident rows)
  struct KP { int toff, rd, sd, tile; unsigned koff; bool hi; };
  int cur_r = 0, cur_s = 0, cur_cc = 0, cur_tile = 0;
  auto next_kp = [&]() {
    KP k;
    const int c0 = cur_cc * 64;
    k.rd = cur_r * a.dil;
    k.sd = cur_s * a.dil;
    k.koff = (unsigned)(((cur_r * a.KW + cur_s) * a.C + c0) * ES);
    k.hi = DUAL && c0 >= a.C1;
    k.toff = k.hi ? (k.rd * a.W + k.sd) * a.ldx2 + (c0 - a.C1) : (k.rd * a.W + k.sd) * a.ldx + c0;
    k.tile = cur_tile;
    if (++cur_s == a.KW) {
      cur_s = 0;
      if (++cur_r == a.KH) {
        cur_r = 0;
        if (++cur_cc * 64 >= a.C) { cur_cc = 0; ++cur_tile; }
      }
    }
    return k;
  };
  auto stage_p = [&](const KP& k, int slot, int ph) {
    if (k.tile != meta_tile) rows_for(k.tile);  // halves are staged in stream order: switch once per tile
    const unsigned dst = lds0 + slot * PP_SLOT + ph * PP_HALF + (16 * wid) * 128;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bool ok = mok[ph][q];
      if (PADCHK)
        ok = ok && (unsigned)(h0[ph][q] + k.rd) < (unsigned)a.H && (unsigned)(w0[ph][q] + k.sd) < (unsigned)a.W;
      const unsigned vo = ok ? (unsigned)(((k.hi ? b2[ph][q] : b1[ph][q]) + k.toff) * ES) : BUF_OOB;
      if (DUAL) dma16u(k.hi ? rx2 : rx, vo, 0, dst + q * 8 * 128);
      else dma16(rx, vo, 0, dst + q * 8 * 128);
    }
  };
  auto stage_c = [&](const KP& k, int slot, int ch) {
    if (k.tile != meta_tile) rows_for(k.tile);
    const unsigned dst = lds0 + slot * PP_SLOT + (2 + ch) * PP_HALF + (16 * wid) * 128;
#pragma unroll
    for (int q = 0; q < 2; ++q) dma16(rw, vb[ch][q], k.koff, dst + q * 8 * 128);
  };

  // timing ablation, diagnostic builds only (-DDMF_PP_ABLATE=<bits>, tools/pp_ablate.sh; results are garbage
  // when any bit is set): bit 1 skips the steady state's vmcnt waits, bit 2 its LDS-DMA issue, bit 4 its
  // fragment reads, bit 8 its MFMAs. A compile-time constant (a run-time mask changes the register
  // allocation and spills); in the product build it is 0.
#ifdef DMF_PP_ABLATE
  constexpr int dbg = DMF_PP_ABLATE;  // one diagnostic library per bit set
#else
  constexpr int dbg = 0;
#endif
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  uint4 pv[2][4], cv0[2][2], cv1[2][2];  // [k32 half][fragment]
  auto read_p = [&](const char* slot, int ph) {
    const char* base = slot + ph * PP_HALF;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int rho = 64 * wm + 16 * ii + fr, ch = kk * 4 + fg;
        pv[kk][ii] = *(const uint4*)(base + rho * 128 + ((ch ^ (rho & 7)) << 4));
      }
  };
  auto read_c = [&](const char* slot, int chh, uint4 (&cv)[2][2]) {
    const char* base = slot + (2 + chh) * PP_HALF;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j0 = 0; j0 < 2; ++j0) {
        const int rho = 32 * wn + 16 * j0 + fr, ch = kk * 4 + fg;
        cv[kk][j0] = *(const uint4*)(base + rho * 128 + ((ch ^ (rho & 7)) << 4));
      }
  };
  // one output quadrant over K 64: pixel frags 4*ph .. +3, channel frags 2*ch, 2*ch + 1
  auto mma_q = [&](int ph, const uint4 (&cv)[2][2], int chh) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j0 = 0; j0 < 2; ++j0)
          acc[4 * ph + ii][2 * chh + j0] = mfma16<T>(cv[kk][j0], pv[kk][ii], acc[4 * ph + ii][2 * chh + j0]);
  };
  // the MFMA segment of phase p: barrier, this wave's fragment reads retired, 16 MFMAs at priority 1, barrier
  auto mfma_segment = [&](int p) {
    __builtin_amdgcn_sched_barrier(0);
    pp_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if (dbg & 8) {
    } else if (p == 0) mma_q(0, cv0, 0);
    else if (p == 1) mma_q(0, cv1, 1);
    else if (p == 2) mma_q(1, cv1, 1);
    else mma_q(1, cv0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    pp_barrier();
  };
  // the finished tile's epilogue: realign the two wave groups (the statistics combine has barriers),
  // store / reduce from the accumulators (ps_epilogue zeroes them), re-stagger
  auto epilogue = [&](int j, bool restagger) {
    if (wm == 0) pp_barrier();
    ps_epilogue<EPI, QBN, 8, QBM, T>(a, acc, tile_lin(j), ry, sred, sbias, tid, wm, wn, fr, fg);
    __builtin_amdgcn_sched_barrier(0);
    if (restagger && wm == 1) pp_barrier();
  };

  // prologue: P0 C0 C1 P1 of K-tile 0, P0 C0 of K-tile 1 -- issue order == consumption order
  KP k1 = next_kp();  // K-tile 0
  stage_p(k1, 0, 0); stage_c(k1, 0, 0); stage_c(k1, 0, 1); stage_p(k1, 0, 1);
  KP k2 = k1;
  if (G > 1) {
    k1 = next_kp();  // K-tile 1
    stage_p(k1, 1, 0); stage_c(k1, 1, 0);
    vm_wait<8>();  // this wave's pieces of P0(0), C0(0) landed
  } else {
    vm_wait<4>();
  }
  if (G > 2) k2 = next_kp();  // K-tile 2
  pp_barrier();  // ... and every wave's, before the leading group's first reads
  __builtin_amdgcn_sched_barrier(0);
  if (wm == 1) pp_barrier();  // the stagger: waves 4-7 run one barrier interval behind

  // one K-tile g of the steady state (K-tiles g+1 = k1 and g+2 = k2 exist). After an epilogue its
  // stores (16 per wave, +2 atomics) are younger than this K-tile's halves: the waits count 16 more.
  int g = 0, kt = 0, j = 0;
  bool after_epi = false;
  for (; g + 2 < G; ++g) {
    const char* slot = smem + (g & 1) * PP_SLOT;
    const int s1 = (g + 1) & 1, s2 = g & 1;
    if (!(dbg & 4)) { read_p(slot, 0); read_c(slot, 0, cv0); }
    if (!(dbg & 2)) stage_c(k1, s1, 1);
    if (!(dbg & 1)) { if (after_epi) vm_wait<24>(); else vm_wait<8>(); }  // C1(g) landed
    mfma_segment(0);
    if (!(dbg & 4)) read_c(slot, 1, cv1);
    if (!(dbg & 2)) stage_p(k1, s1, 1);
    if (!(dbg & 1)) { if (after_epi) vm_wait<24>(); else vm_wait<8>(); }  // P1(g)
    mfma_segment(1);
    if (!(dbg & 4)) read_p(slot, 1);
    if (!(dbg & 2)) stage_p(k2, s2, 0);
    if (!(dbg & 1)) { if (after_epi) vm_wait<26>(); else vm_wait<10>(); }
    mfma_segment(2);
    if (!(dbg & 2)) stage_c(k2, s2, 0);
    if (!(dbg & 1)) { if (after_epi) vm_wait<24>(); else vm_wait<8>(); }  // P0(g+1), C0(g+1)
    mfma_segment(3);
    after_epi = false;
    k1 = k2;
    if (g + 3 < G) k2 = next_kp();
    if (++kt == nk) {
      epilogue(j, true);
      kt = 0;
      ++j;
      after_epi = true;
    }
  }
  // the last two K-tiles of the stream: stage what remains, drain every wait
  for (; g < G; ++g) {
    const char* slot = smem + (g & 1) * PP_SLOT;
    const bool more = g + 1 < G;
    read_p(slot, 0); read_c(slot, 0, cv0);
    if (more) stage_c(k1, (g + 1) & 1, 1);
    vm_wait<0>();
    mfma_segment(0);
    read_c(slot, 1, cv1);
    if (more) stage_p(k1, (g + 1) & 1, 1);
    vm_wait<0>();
    mfma_segment(1);
    read_p(slot, 1);
    vm_wait<0>();
    mfma_segment(2);
    vm_wait<0>();
    mfma_segment(3);
    if (++kt == nk) {
      epilogue(j, g + 1 < G);
      kt = 0;
      ++j;
    }
  }
}

static int g_pp_persist = 1;  // dmf_conv_tune key 8: 1 persistent grid (<= one block per CU), 0 one block per tile

int conv_pp_tune(int value) {
  g_pp_persist = value;
  return 0;
}


int launch_conv_pp(ConvArgs& a, int epi, bool plain, size_t lds_bias, hipStream_t st, int dtype) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  const int ntile = a.mtiles * a.ntiles;
  const dim3 g((unsigned)(g_pp_persist ? std::min(ntile, ncu) : ntile)), b(PP_THREADS);
  const size_t lds = (size_t)PP_LDS + lds_bias;
  DMF_CHECK_ARG(lds <= 160 * 1024, "conv_pp: %d output channels of bias exceed the LDS staging", a.Nout);
  a.dbg = 0;
#define DMF_PP(E, TT)                                                                                    \
  do {                                                                                                   \
    if (a.x2 != nullptr) hipLaunchKernelGGL((k_conv_fwd_pp<true, true, E, TT>), g, b, lds, st, a);      \
    else if (plain) hipLaunchKernelGGL((k_conv_fwd_pp<false, false, E, TT>), g, b, lds, st, a);         \
    else hipLaunchKernelGGL((k_conv_fwd_pp<true, false, E, TT>), g, b, lds, st, a);                     \
  } while (0)
#define DMF_PP_E(TT)                  \
  do {                                \
    switch (epi) {                    \
      case 0: DMF_PP(0, TT); break;   \
      case 1: DMF_PP(1, TT); break;   \
      case 2: DMF_PP(2, TT); break;   \
      case 3: DMF_PP(3, TT); break;   \
      case 5: DMF_PP(5, TT); break;   \
      default: DMF_PP(4, TT); break;  \
    }                                 \
  } while (0)
  if (dtype == DMF_F16) DMF_PP_E(f16_t);
  else DMF_PP_E(bf16_t);
#undef DMF_PP_E
#undef DMF_PP
  DMF_LAUNCH_CHECK("conv_pp");
  return 0;
}

}  // namespace dmf
