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
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
}
// wait until at most 2*younger LDS-DMA pieces of this wave are in flight (uniform)
__device__ __forceinline__ void vm_wait_halves(int younger) {
  switch (younger) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<2>(); break;
    case 2: vm_wait<4>(); break;
    case 3: vm_wait<6>(); break;
    case 4: vm_wait<8>(); break;
    default: vm_wait<10>(); break;
  }
}

template <bool PADCHK, bool DUAL, int EPI>
__global__ void __launch_bounds__(PP_THREADS, 1) k_conv_fwd_pp(ConvArgs a) {
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
  if (a.bias) {
    for (int i = tid; i < a.Nout; i += PP_THREADS) sbias[i] = a.bias[i];
    __syncthreads();
  }

  const v4i_t rx = buf_rsrc(a.x, (long long)a.N * a.H * a.W * a.ldx * ES);
  const v4i_t rx2 = buf_rsrc(DUAL ? a.x2 : a.x, (long long)a.N * a.H * a.W * (DUAL ? a.ldx2 : a.ldx) * ES);
  const v4i_t rw = buf_rsrc(a.w, (long long)a.Nout * a.Ktot * ES);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)((long long)a.M * a.ldy * ES), BUF_FLAGS);
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lin / a.ntiles, nt = lin - (lin / a.ntiles) * a.ntiles;
  const int m0 = mt * 256, n0 = nt * 256;
  const int nk = a.Ktot / 64;
  const int taps = a.KH * a.KW;
  const int hw = a.Ho * a.Wo;

  // staging rows of this lane: piece q (0, 1) of a half covers half rows 16*wid + 8*q + (0..7)
  int h0[2][2], w0[2][2], b1[2][2], b2[2][2];
  bool mok[2][2];
  unsigned vb[2][2];
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

  // K-tile kt: channel chunk outer, filter tap inner (the taps of one chunk re-read L2-resident rows)
  auto stage_p = [&](int kt, int ph) {
    const int cc = kt / taps, tap = kt - cc * taps;
    const int r = tap / a.KW, s = tap - r * a.KW;
    const int c0 = cc * 64, rd = r * a.dil, sd = s * a.dil;
    const bool hi = DUAL && c0 >= a.C1;
    const int toff = hi ? (rd * a.W + sd) * a.ldx2 + (c0 - a.C1) : (rd * a.W + sd) * a.ldx + c0;
    const unsigned dst = lds0 + (kt & 1) * PP_SLOT + ph * PP_HALF + (16 * wid) * 128;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bool ok = mok[ph][q];
      if (PADCHK) ok = ok && (unsigned)(h0[ph][q] + rd) < (unsigned)a.H && (unsigned)(w0[ph][q] + sd) < (unsigned)a.W;
      const unsigned vo = ok ? (unsigned)(((hi ? b2[ph][q] : b1[ph][q]) + toff) * ES) : BUF_OOB;
      dma16u(hi ? rx2 : rx, vo, 0, dst + q * 8 * 128);
    }
  };
  auto stage_c = [&](int kt, int ch) {
    const int cc = kt / taps, tap = kt - cc * taps;
    const unsigned koff = (unsigned)((tap * a.C + cc * 64) * ES);
    const unsigned dst = lds0 + (kt & 1) * PP_SLOT + (2 + ch) * PP_HALF + (16 * wid) * 128;
#pragma unroll
    for (int q = 0; q < 2; ++q) dma16u(rw, vb[ch][q], koff, dst + q * 8 * 128);
  };

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
          acc[4 * ph + ii][2 * chh + j0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              *(const bf16x8_t*)&cv[kk][j0], *(const bf16x8_t*)&pv[kk][ii], acc[4 * ph + ii][2 * chh + j0], 0, 0, 0);
  };

  // prologue: P0 C0 C1 P1 of K-tile 0, P0 C0 of K-tile 1 -- issue order == consumption order
  int issued = 0;
  stage_p(0, 0); stage_c(0, 0); stage_c(0, 1); stage_p(0, 1);
  issued = 4;
  if (nk > 1) { stage_p(1, 0); stage_c(1, 0); issued = 6; }
  vm_wait_halves(issued - 1 - 1);  // this wave's pieces of P0(0), C0(0) landed
  pp_barrier();                    // ... and every wave's, before the leading group's first reads
  __builtin_amdgcn_sched_barrier(0);
  if (wm == 1) pp_barrier();  // the stagger: waves 4-7 run one barrier interval behind

  for (int t = 0; t < nk; ++t) {
    const char* slot = smem + (t & 1) * PP_SLOT;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // ---- LOAD segment: this phase's fragments, one half-tile of staging, the counted wait
      if (p == 0) { read_p(slot, 0); read_c(slot, 0, cv0); }
      else if (p == 1) read_c(slot, 1, cv1);
      else if (p == 2) read_p(slot, 1);
      if (p == 0 && t + 1 < nk) { stage_c(t + 1, 1); ++issued; }
      if (p == 1 && t + 1 < nk) { stage_p(t + 1, 1); ++issued; }
      if (p == 2 && t + 2 < nk) { stage_p(t + 2, 0); ++issued; }
      if (p == 3 && t + 2 < nk) { stage_c(t + 2, 0); ++issued; }
      // the half the NEXT phase reads: C1(t), P1(t), (nothing new), P0/C0(t+1) -> sequence index
      const int need = p == 0 ? 4 * t + 2 : (p == 1 || p == 2) ? 4 * t + 3 : 4 * t + 5;
      vm_wait_halves(max(0, min(issued - 1 - need, 5)));
      __builtin_amdgcn_sched_barrier(0);
      pp_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // ---- MFMA segment
      __builtin_amdgcn_s_setprio(1);
      if (p == 0) mma_q(0, cv0, 0);
      else if (p == 1) mma_q(0, cv1, 1);
      else if (p == 2) mma_q(1, cv1, 1);
      else mma_q(1, cv0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      pp_barrier();
    }
  }
  if (wm == 0) pp_barrier();  // realign the two wave groups for the epilogue's barriers
  ps_epilogue<EPI>(a, acc, lin, ry, sred, sbias, tid, wm, wn, fr, fg);
}

int launch_conv_pp(ConvArgs& a, int epi, bool plain, size_t lds_bias, hipStream_t st) {
  const dim3 g((unsigned)(a.mtiles * a.ntiles)), b(PP_THREADS);
  const size_t lds = (size_t)PP_LDS + lds_bias;
  DMF_CHECK_ARG(lds <= 160 * 1024, "conv_pp: %d output channels of bias exceed the LDS staging", a.Nout);
  a.dbg = 0;
#define DMF_PP(E)                                                                                    \
  do {                                                                                               \
    if (a.x2 != nullptr) hipLaunchKernelGGL((k_conv_fwd_pp<true, true, E>), g, b, lds, st, a);      \
    else if (plain) hipLaunchKernelGGL((k_conv_fwd_pp<false, false, E>), g, b, lds, st, a);         \
    else hipLaunchKernelGGL((k_conv_fwd_pp<true, false, E>), g, b, lds, st, a);                     \
  } while (0)
  switch (epi) {
    case 0: DMF_PP(0); break;
    case 1: DMF_PP(1); break;
    case 2: DMF_PP(2); break;
    case 3: DMF_PP(3); break;
    default: DMF_PP(4); break;
  }
#undef DMF_PP
  DMF_LAUNCH_CHECK("conv_pp");
  return 0;
}

}  // namespace dmf
