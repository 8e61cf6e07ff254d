// Fused attention forward of the token blocks (transformer_model.py:100-116 MultiHeadSelfAttention,
// the TransformerStage / ViT blocks) for a forward that builds no autograd graph (frozen encoders,
// mode A): o = dropout(softmax(q k^T * scale)) v per (batch item, head), with key padding (keys >= nv
// masked) and the Philox attention dropout of k_softmax_drop (element index row * n + key, row =
// (b * heads + h) * n + query), in one launch that never writes the [b*h, n, n] scores or
// probabilities -- the unfused path (QK^T GEMM to fp32 scores, k_softmax_drop, PV GEMM) moves
// ~0.5 GB per layer at 576 tokens.
//
// Block = 64 queries of one (b, h), 4 waves of 16 queries; the keys stream through two LDS stages of
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

constexpr int FA_D = 128, FA_QT = 64, FA_KT = 64, FA_THREADS = 256;
constexpr int FA_TILE = FA_KT * FA_D * 2;  // one 64-key x 128-d bf16 tile: 256-B rows
constexpr int FA_STAGE = 2 * FA_TILE;      // K + V
typedef short fa_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) fa_v4s fa_lds_v4s;
typedef __attribute__((ext_vector_type(8))) short fa_v8s;

// byte offset of logical 16-B chunk `ch` of row `row` (conv_wgrad.hip wtr_off: chunk XOR over the row's
// low 4 bits, conflict-free for both the 16-row b128 reads and the transposed b64 reads)
__device__ __forceinline__ int fa_off(int row, int ch) {
  return (row << 8) + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

__global__ void __launch_bounds__(FA_THREADS, 2)
    k_flash_attn_fwd(const bf16_t* __restrict__ qkv, int ldq, long long nrows, int E, int heads, int n, int nv,
                     float scale_log2, float dp, const unsigned long long* rng, int site, bf16_t* __restrict__ o,
                     int ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, bi = bh / heads, hd = bh - bi * heads;
  const int fr = lane & 15, g = lane >> 4;
  const int qrow = blockIdx.x * FA_QT + wid * 16 + fr;  // this lane's query (within the sequence)
  const long long rbase = (long long)bi * n;             // token row of (bi, 0)
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const v4i_t rq = buf_rsrc(qkv, nrows * ldq * 2);

  // Q^T fragments (the 16-column operand): query qrow, head dims 32 ks + 8 g .. +7
  uint4 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    qf[ks] = qrow < n ? *(const uint4*)(qkv + (rbase + qrow) * ldq + hd * FA_D + 32 * ks + 8 * g)
                      : make_uint4(0, 0, 0, 0);

  // K / V tile of keys k0 .. k0 + 63 into stage `stage`: 16 DMA pieces of 4 rows per tensor, 4 per wave
  auto issue = [&](int stage, int k0) {
    const unsigned S = lds0 + stage * FA_STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int P = wid * 4 + i;
      const int row = 4 * P + (lane >> 4);
      const int ch = (lane & 15) ^ (((lane >> 4) << 2) | (P & 3));  // logical chunk landing in slot lane & 15
      const int key = k0 + row;
      const unsigned kb =
          key < n ? (unsigned)(((rbase + key) * ldq + E + hd * FA_D + ch * 8) * 2) : BUF_OOB;
      dma16(rq, kb, 0, S + P * 1024);
      dma16(rq, key < n ? kb + (unsigned)(E * 2) : BUF_OOB, 0, S + FA_TILE + P * 1024);
    }
  };

  dmf_f32x4 oacc[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) oacc[f] = dmf_f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  const float ks_drop = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  const unsigned long long drow = ((unsigned long long)bh * n + (unsigned)qrow) * (unsigned long long)n;
  const int q = (lane >> 2) & 3, p4 = lane & 3;
  const int nkt = (nv + FA_KT - 1) / FA_KT;
  issue(0, 0);
  for (int kt = 0; kt < nkt; ++kt) {
    // this stage's DMA (the only one in flight) retired; the barrier publishes every wave's pieces and
    // orders the refill of the other stage after every wave's reads of tile kt - 1
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 1 < nkt) issue((kt + 1) & 1, (kt + 1) * FA_KT);
    const char* SK = smem + (kt & 1) * FA_STAGE;
    const char* SV = SK + FA_TILE;
    // S^T = K Q^T: s[f][r] = score(key kt*64 + 16 f + 4 g + r, query qrow)
    dmf_f32x4 s[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      s[f] = dmf_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        s[f] = mfma16<bf16_t>(*(const uint4*)(SK + fa_off(16 * f + fr, 4 * kk + g)), qf[kk], s[f]);
    }
    // online softmax of query qrow over this lane's 16 keys (+ the 3 other lanes of the same query)
    const int kb0 = kt * FA_KT + 4 * g;
    float t[16];
    float mt = -INFINITY;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        t[4 * f + r] = kb0 + 16 * f + r < nv ? s[f][r] * scale_log2 : -INFINITY;
        mt = fmaxf(mt, t[4 * f + r]);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);
    m = mn;
    lsum *= alpha;
#pragma unroll
    for (int f = 0; f < 8; ++f) oacc[f] *= alpha;
    uint32_t pp[4][2];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      float p[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = exp2f(t[4 * f + r] - mn);
        lsum += p[r];
      }
      if (dp > 0.f) {
        bool keep[4];
        dropout_keep4(rng, site, drow + (unsigned long long)(kb0 + 16 * f), dp, keep);
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = keep[r] ? p[r] * ks_drop : 0.f;
      }
      pp[f][0] = B16<bf16_t>::pack(p[0], p[1]);
      pp[f][1] = B16<bf16_t>::pack(p[2], p[3]);
    }
    // O^T += V^T P^T over the tile's two 32-key steps
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      // P^T operand: query qrow, keys 32 st + 8 g .. +7 = rows 8 (g & 1) .. +7 of key fragment 2 st + g / 2,
      // held by lane groups 2 (g & 1) and 2 (g & 1) + 1 of the same query
      const int src0 = ((2 * (g & 1)) << 4) | fr, src1 = src0 + 16;
      const uint32_t a0 = __shfl(pp[2 * st][0], src0, 64), a1 = __shfl(pp[2 * st][1], src0, 64);
      const uint32_t b0 = __shfl(pp[2 * st][0], src1, 64), b1 = __shfl(pp[2 * st][1], src1, 64);
      const uint32_t c0 = __shfl(pp[2 * st + 1][0], src0, 64), c1 = __shfl(pp[2 * st + 1][1], src0, 64);
      const uint32_t d0 = __shfl(pp[2 * st + 1][0], src1, 64), d1 = __shfl(pp[2 * st + 1][1], src1, 64);
      const uint4 pb = g < 2 ? make_uint4(a0, a1, b0, b1) : make_uint4(c0, c1, d0, d1);
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
        oacc[fd] = mfma16<bf16_t>(__builtin_bit_cast(uint4, af), pb, oacc[fd]);
      }
    }
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (qrow >= n) return;
  const float inv = 1.f / lsum;
  bf16_t* dst = o + (rbase + qrow) * ldo + hd * FA_D + 4 * g;
#pragma unroll
  for (int fd = 0; fd < 8; ++fd) {
    uint2 w;
    w.x = B16<bf16_t>::pack(oacc[fd][0] * inv, oacc[fd][1] * inv);
    w.y = B16<bf16_t>::pack(oacc[fd][2] * inv, oacc[fd][3] * inv);
    *(uint2*)(dst + 16 * fd) = w;
  }
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
  const dim3 grid((unsigned)cdiv(n, FA_QT), (unsigned)(batch * heads));
  DMF_CHECK_ARG(batch * heads < 65536, "dmf_flash_attn_fwd: batch x heads too large");
  hipLaunchKernelGGL(k_flash_attn_fwd, grid, dim3(FA_THREADS), 2 * FA_STAGE, (hipStream_t)stream,
                     (const bf16_t*)qkv, ldq, (long long)batch * n, E, heads, n, nv, scale * 1.4426950408889634f,
                     dropout_p, rng, site, (bf16_t*)o, ldo);
  DMF_LAUNCH_CHECK("dmf_flash_attn_fwd");
  return 0;
}

}  // namespace dmf
