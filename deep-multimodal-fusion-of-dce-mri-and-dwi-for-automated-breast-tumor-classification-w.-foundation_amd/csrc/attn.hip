// Fused attention forward of the token blocks (transformer_model.py:100-116 MultiHeadSelfAttention,
// the TransformerStage / ViT blocks) for a forward that builds no autograd graph (frozen encoders,
// mode A): o = dropout(softmax(q k^T * scale)) v per (batch item, head), with key padding (keys >= nv
// masked) and the Philox attention dropout of k_softmax_drop (element index row * n + key, row =
// (b * heads + h) * n + query), in one launch that never writes the [b*h, n, n] scores or
// probabilities -- the unfused path (QK^T GEMM to fp32 scores, k_softmax_drop, PV GEMM) moves
// ~0.5 GB per layer at 576 tokens.
//
// Block = 64 * NQ queries of one (b, h), 4 waves of 16 * NQ queries; the keys stream through two LDS stages of
// 64 keys (K and V tiles, 64 x 128 bf16 each, LDS-DMA with the source-side XOR swizzle of
// conv_wgrad.hip's transposed-read layout). Per key tile a wave computes S^T = K Q^T (keys as the
// 16-row MFMA operand, so a lane holds 4 consecutive keys of ONE query: the row max / sum are lane-local
// plus two shuffles, the dropout mask is one Philox block per 4 keys, and the online-softmax rescale
// touches only that lane's own O accumulators), the online softmax in the exp2 domain, then
// O^T += V^T P^T (V^T fragments by ds_read_b64_tr_b16, P^T fragments gathered from the S^T lanes by
// ds_bpermute). The row sum keeps the pre-dropout probabilities (softmax first, dropout after, as the
// reference); o = O / sum at the end, bf16.
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

constexpr int FA_D = 128, FA_QT = 64, FA_THREADS = 256;
typedef short fa_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) fa_v4s fa_lds_v4s;
typedef __attribute__((ext_vector_type(8))) short fa_v8s;

// byte offset of logical 16-B chunk `ch` of row `row` (conv_wgrad.hip wtr_off: chunk XOR over the row's
// low 4 bits, conflict-free for both the 16-row b128 reads and the transposed b64 reads)
__device__ __forceinline__ int fa_off(int row, int ch) {
  return (row << 8) + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// NQ: 16-query fragments per wave (2: each K / V^T fragment read from LDS feeds two MFMAs -- at one
// fragment the loop is bound by the LDS reads, 32 KiB per wave per key tile against 32 MFMAs).
// KT keys per tile (64 or 32), NST LDS stages: the next NST - 1 tiles are in flight while one is
// computed (a tile's compute is shorter than an LDS-DMA round trip under load: with one tile ahead the
// loop waits on the DMA every step).
template <int NQ, int KT, int NST>
__global__ void __launch_bounds__(FA_THREADS, 2)
    k_flash_attn_fwd(const bf16_t* __restrict__ qkv, int ldq, long long nrows, int E, int heads, int n, int nv,
                     float scale_log2, float dp, const unsigned long long* rng, int site, bf16_t* __restrict__ o,
                     int ldo) {
  constexpr int KF = KT / 16;               // 16-key fragments per tile
  constexpr int TILE = KT * FA_D * 2;       // one K (or V) tile: 256-B rows
  constexpr int STAGE = 2 * TILE;
  constexpr int PW = KT / 16;               // 1 KiB DMA pieces per wave per tensor (KT / 4 rows / 4 waves)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, bi = bh / heads, hd = bh - bi * heads;
  const int fr = lane & 15, g = lane >> 4;
  const long long rbase = (long long)bi * n;  // token row of (bi, 0)
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const v4i_t rq = buf_rsrc(qkv, nrows * ldq * 2);
  int qrow[NQ];  // this lane's queries (within the sequence), one per query fragment
#pragma unroll
  for (int j = 0; j < NQ; ++j) qrow[j] = blockIdx.x * (64 * NQ) + (wid * NQ + j) * 16 + fr;

  // Q^T fragments (the 16-column operand): query qrow[j], head dims 32 ks + 8 g .. +7
  uint4 qf[NQ][4];
#pragma unroll
  for (int j = 0; j < NQ; ++j)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      qf[j][ks] = qrow[j] < n ? *(const uint4*)(qkv + (rbase + qrow[j]) * ldq + hd * FA_D + 32 * ks + 8 * g)
                              : make_uint4(0, 0, 0, 0);

  // K / V tile of keys k0 .. k0 + KT - 1 into stage `stage`: KT / 4 DMA pieces of 4 rows per tensor
  auto issue = [&](int stage, int k0) {
    const unsigned S = lds0 + stage * STAGE;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int P = wid * PW + i;
      const int row = 4 * P + (lane >> 4);
      const int ch = (lane & 15) ^ (((lane >> 4) << 2) | (P & 3));  // logical chunk landing in slot lane & 15
      const int key = k0 + row;
      const unsigned kb =
          key < n ? (unsigned)(((rbase + key) * ldq + E + hd * FA_D + ch * 8) * 2) : BUF_OOB;
      dma16(rq, kb, 0, S + P * 1024);
      dma16(rq, key < n ? kb + (unsigned)(E * 2) : BUF_OOB, 0, S + TILE + P * 1024);
    }
  };

  dmf_f32x4 oacc[NQ][8];
#pragma unroll
  for (int j = 0; j < NQ; ++j)
#pragma unroll
    for (int f = 0; f < 8; ++f) oacc[j][f] = dmf_f32x4{0.f, 0.f, 0.f, 0.f};
  float m[NQ], lsum[NQ];
  unsigned long long drow[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    m[j] = -INFINITY;
    lsum[j] = 0.f;
    drow[j] = ((unsigned long long)bh * n + (unsigned)qrow[j]) * (unsigned long long)n;
  }
  const float ks_drop = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  // the Philox (seed, offset) read once (the K loop's barriers would reload them per mask)
  const unsigned long long rseed = dp > 0.f ? rng[0] : 0ull, roff = dp > 0.f ? rng[1] : 0ull;
  const int q = (lane >> 2) & 3, p4 = lane & 3;
  const int nkt = (nv + KT - 1) / KT;
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nkt) issue(t, t * KT);
  for (int kt = 0; kt < nkt; ++kt) {
    // retire tile kt (the younger tiles' 2 * PW pieces per wave each may stay in flight: vmcnt is in
    // order); the barrier publishes every wave's pieces and orders the refill of stage (kt - 1) % NST
    // after every wave's reads of it
    const int ahead = min(NST - 2, nkt - 1 - kt);  // tiles issued after kt and still in flight
    if (NST == 3 && ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * PW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + NST - 1 < nkt) issue((kt + NST - 1) % NST, (kt + NST - 1) * KT);
    const char* SK = smem + (kt % NST) * STAGE;
    const char* SV = SK + TILE;
    // S^T = K Q^T: s[j][f][r] = score(key kt*KT + 16 f + 4 g + r, query qrow[j])
    dmf_f32x4 s[NQ][KF];
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
      for (int f = 0; f < KF; ++f) s[j][f] = dmf_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < KF; ++f)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const uint4 kf = *(const uint4*)(SK + fa_off(16 * f + fr, 4 * kk + g));
#pragma unroll
        for (int j = 0; j < NQ; ++j) s[j][f] = mfma16<bf16_t>(kf, qf[j][kk], s[j][f]);
      }
    // online softmax of each query over this lane's 4 KF keys (+ the 3 other lanes of the same query)
    const int kb0 = kt * KT + 4 * g;
    const bool full = (kt + 1) * KT <= nv;  // (wave-uniform) no padded key in this tile
    uint32_t pp[NQ][KF][2];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      // the max on the raw scores (scale > 0), then exp2(s * scale_log2 - max) as one FMA + exp
      float mt = -INFINITY;
      if (!full) {
#pragma unroll
        for (int f = 0; f < KF; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kb0 + 16 * f + r >= nv) s[j][f][r] = -INFINITY;
      }
#pragma unroll
      for (int f = 0; f < KF; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) mt = fmaxf(mt, s[j][f][r]);
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m[j], mt * scale_log2);
      const float alpha = exp2f(m[j] - mn);
      m[j] = mn;
      lsum[j] *= alpha;
#pragma unroll
      for (int f = 0; f < 8; ++f) oacc[j][f] *= alpha;
#pragma unroll
      for (int f = 0; f < KF; ++f) {
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = exp2f(__builtin_fmaf(s[j][f][r], scale_log2, -mn));
          lsum[j] += p[r];
        }
        if (dp > 0.f) {
          bool keep[4];
          dropout_keep4v(rseed, roff, site, drow[j] + (unsigned long long)(kb0 + 16 * f), dp, keep);
#pragma unroll
          for (int r = 0; r < 4; ++r) p[r] = keep[r] ? p[r] * ks_drop : 0.f;
        }
        pp[j][f][0] = B16<bf16_t>::pack(p[0], p[1]);
        pp[j][f][1] = B16<bf16_t>::pack(p[2], p[3]);
      }
    }
    // O^T += V^T P^T over the tile's 32-key steps
#pragma unroll
    for (int st = 0; st < KT / 32; ++st) {
      // P^T operand: query qrow[j], keys 32 st + 8 g .. +7 = rows 8 (g & 1) .. +7 of key fragment
      // 2 st + g / 2, held by lane groups 2 (g & 1) and 2 (g & 1) + 1 of the same query
      const int src0 = ((2 * (g & 1)) << 4) | fr, src1 = src0 + 16;
      uint4 pb[NQ];
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const uint32_t a0 = __shfl(pp[j][2 * st][0], src0, 64), a1 = __shfl(pp[j][2 * st][1], src0, 64);
        const uint32_t b0 = __shfl(pp[j][2 * st][0], src1, 64), b1 = __shfl(pp[j][2 * st][1], src1, 64);
        const uint32_t c0 = __shfl(pp[j][2 * st + 1][0], src0, 64), c1 = __shfl(pp[j][2 * st + 1][1], src0, 64);
        const uint32_t d0 = __shfl(pp[j][2 * st + 1][0], src1, 64), d1 = __shfl(pp[j][2 * st + 1][1], src1, 64);
        pb[j] = g < 2 ? make_uint4(a0, a1, b0, b1) : make_uint4(c0, c1, d0, d1);
      }
#pragma unroll
      for (int fd = 0; fd < 8; ++fd) {
        fa_v8s af;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int key = 32 * st + 8 * g + 4 * h + q;
          const fa_v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (fa_lds_v4s*)(SV + fa_off(key, 2 * fd + (p4 >> 1)) + 8 * (p4 & 1)));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[4 * h + e] = v[e];
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) oacc[j][fd] = mfma16<bf16_t>(__builtin_bit_cast(uint4, af), pb[j], oacc[j][fd]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    float l = lsum[j];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qrow[j] >= n) continue;
    const float inv = 1.f / l;
    bf16_t* dst = o + (rbase + qrow[j]) * ldo + hd * FA_D + 4 * g;
#pragma unroll
    for (int fd = 0; fd < 8; ++fd) {
      uint2 w;
      w.x = B16<bf16_t>::pack(oacc[j][fd][0] * inv, oacc[j][fd][1] * inv);
      w.y = B16<bf16_t>::pack(oacc[j][fd][2] * inv, oacc[j][fd][3] * inv);
      *(uint2*)(dst + 16 * fd) = w;
    }
  }
}

// dmf_flash_attn_tune: 1 = one query fragment per wave, 64-key tiles, 2 stages; 2 (default) = two
// fragments, 64-key tiles, 2 stages; 3 = two fragments, 32-key tiles, 3 stages (two tiles in flight).
// Measured (tools/gemm_bench.py, 32 x 576 tokens, E = 512, 4 heads; profiles/r05i_flash_attn.txt):
// 77.4 / 67.7 / 79.0 us without dropout, 108.9 / 107.6 / 120.4 us with p = 0.1 (the unfused path:
// 64.4 + 58.0 + 67.4 = 190 us) -- more keys in flight buys nothing, the Philox masks cost ~40 us
static int g_fa_var = 2;
extern "C" int dmf_flash_attn_tune(int var) {
  DMF_CHECK_ARG(var >= 1 && var <= 3, "dmf_flash_attn_tune: variant %d (1..3)", var);
  g_fa_var = var;
  return 0;
}

extern "C" int dmf_flash_attn_fwd(const void* qkv, int ldq, int batch, int n, int nv, int E, int heads, float scale,
                                  float dropout_p, const unsigned long long* rng, int site, void* o, int ldo,
                                  void* stream) {
  DMF_CHECK_ARG(qkv && o && batch > 0 && n > 0 && heads > 0 && E == heads * FA_D,
                "dmf_flash_attn_fwd: head dim must be %d (E=%d, heads=%d)", FA_D, E, heads);
  DMF_CHECK_ARG(nv >= 1 && nv <= n, "dmf_flash_attn_fwd: valid length %d must be in [1, n=%d]", nv, n);
  DMF_CHECK_ARG(ldq >= 3 * E && ldq % 8 == 0 && ldo >= E && ldo % 4 == 0 && ((uintptr_t)qkv % 16) == 0 &&
                    ((uintptr_t)o % 8) == 0,
                "dmf_flash_attn_fwd: row strides / alignment (ldq=%d ldo=%d)", ldq, ldo);
  DMF_CHECK_ARG((long long)batch * n * ldq * 2 < (1LL << 31), "dmf_flash_attn_fwd: qkv exceeds 2 GiB");
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_flash_attn_fwd: dropout needs rng state");
  DMF_CHECK_ARG(dropout_p < 1.f, "dmf_flash_attn_fwd: p must be < 1");
  // dropout_keep4v draws one Philox block per 4 consecutive elements of (bh*n + q)*n + key: the
  // element index must stay 4-aligned for the masks to equal dmf_softmax_dropout's
  DMF_CHECK_ARG(dropout_p <= 0.f || n % 4 == 0, "dmf_flash_attn_fwd: dropout needs n %% 4 == 0 (n=%d)", n);
  DMF_CHECK_ARG(batch * heads < 65536, "dmf_flash_attn_fwd: batch x heads too large");
  const int nq = g_fa_var == 1 ? 1 : 2;
  const dim3 grid((unsigned)cdiv(n, FA_QT * nq), (unsigned)(batch * heads));
  const float sl2 = scale * 1.4426950408889634f;
#define DMF_FA(NQ_, KT_, NST_)                                                                                  \
  hipLaunchKernelGGL((k_flash_attn_fwd<NQ_, KT_, NST_>), grid, dim3(FA_THREADS), (size_t)NST_ * KT_ * FA_D * 4, \
                     (hipStream_t)stream, (const bf16_t*)qkv, ldq, (long long)batch * n, E, heads, n, nv, sl2,      \
                     dropout_p, rng, site, (bf16_t*)o, ldo)
  if (g_fa_var == 1) DMF_FA(1, 64, 2);
  else if (g_fa_var == 2) DMF_FA(2, 64, 2);
  else DMF_FA(2, 32, 3);
#undef DMF_FA
  DMF_LAUNCH_CHECK("dmf_flash_attn_fwd");
  return 0;
}

}  // namespace dmf
