// The fusion step's criteria (train_fusion.py:239-296) as fused
// loss + gradient kernels. Each forward writes the scalar loss AND the
// gradient w.r.t. its inputs for a unit upstream gradient; the autograd
// backward rescales it by the incoming grad (dmf_scale_by).
//   focal : LabelSmoothing (loss.py:190-213) -> SoftWeightedFocalLoss
//           (loss.py:157-187), class weights from selector_helpers.py:25-41
//   dice  : SoftDiceLoss (loss.py:45-62) via safe_mask_loss
//           (train_fusion.py:747-760)
//   recon : compute_recon_list_loss (train_fusion.py:709-744) with
//           recon_image_loss/charbonnier (train.py:1041-1048): bilinear
//           32->S upsample, sigmoid, clamp, sqrt((p-t)^2 + 1e-6) against the
//           clamped channel mean of the input -- the SxS upsampled map is never
//           materialised
//   mimic : mimic_feat_loss (train.py:1033-1038) over batch items (Q5)
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

// one block; B rows, K <= 64 classes. Targets: dense soft targets [B][K]
// (LabelSmoothing output) if given, else int64 labels (one-hot, optionally
// smoothed in-kernel). reduction: 0 mean, 1 sum, 2 none (per_row only).
// dlogits: gradient of the reduced loss (per-row loss for 'none').
__global__ void k_focal(const float* __restrict__ logits, const long long* __restrict__ labels,
                        const float* __restrict__ soft, int B, int K, float smoothing, int smooth,
                        const float* __restrict__ cw, float gamma, int reduction, float* __restrict__ loss,
                        float* __restrict__ per_row, float* __restrict__ dlogits) {
  __shared__ float red[16];
  float acc = 0.f;
  const float rscale = reduction == 0 ? 1.f / (float)B : 1.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float* z = logits + (size_t)b * K;
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, z[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(z[k] - mx);
    const float lse = mx + logf(se);
    const long long y = labels ? labels[b] : -1;
    // l = -sum_k t_k w_k (1-p_k)^g logp_k ; dl/dlogp_k = -t_k w_k [(1-p)^g - g (1-p)^(g-1) p logp]
    // dlogp_k/dz_j = delta_kj - p_j
    float row = 0.f, gsum = 0.f;
    float gk[64];
    for (int k = 0; k < K; ++k) {
      const float lp = z[k] - lse;
      const float p = expf(lp);
      float t;
      if (soft) t = soft[(size_t)b * K + k];
      else t = smooth ? (k == y ? 1.f - smoothing : smoothing / (float)(K - 1)) : (k == y ? 1.f : 0.f);
      const float w = cw ? cw[k] : 1.f;
      const float om = fmaxf(1.f - p, 0.f);
      const float fw = powf(om, gamma);
      row += -t * w * fw * lp;
      const float dfw = gamma > 0.f && om > 0.f ? gamma * powf(om, gamma - 1.f) : 0.f;
      const float g = -t * w * (fw - dfw * p * lp);
      gk[k] = g;
      gsum += g;
    }
    acc += row;
    if (per_row) per_row[b] = row;
    if (dlogits) {
      for (int j = 0; j < K; ++j) {
        const float pj = expf(z[j] - lse);
        dlogits[(size_t)b * K + j] = (gk[j] - pj * gsum) * rscale;
      }
    }
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0 && loss) loss[0] = acc * rscale;
}

// LabelSmoothing (loss.py:190-213): fill smoothing/(K-1), label -> 1-smoothing
__global__ void k_label_smooth(const long long* __restrict__ labels, int B, int K, float smoothing,
                               float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * K) return;
  const int b = i / K, k = i % K;
  out[i] = labels[b] == k ? 1.f - smoothing : smoothing / (float)(K - 1);
}

// soft dice over [B][P] logits, target [B][P]; block per sample writes its dice,
// then the last kernel forms the mean. grad: d/dx of 1 - mean_b dice_b
template <typename T, typename TT>
__global__ void k_dice_sums(const T* __restrict__ x, const TT* __restrict__ t, int P, float* __restrict__ sums) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  float si = 0.f, sp = 0.f, st_ = 0.f;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const float p = sigmoid_f(ld(x + (size_t)b * P + i));
    const float tv = ld(t + (size_t)b * P + i);
    si += p * tv;
    sp += p;
    st_ += tv;
  }
  si = block_sum(si, red);
  sp = block_sum(sp, red);
  st_ = block_sum(st_, red);
  if (threadIdx.x == 0) {
    sums[3 * b] = si;
    sums[3 * b + 1] = sp;
    sums[3 * b + 2] = st_;
  }
}

template <typename T, typename TT>
__global__ void k_dice_grad(const T* __restrict__ x, const TT* __restrict__ t, int B, int P, float eps,
                            const float* __restrict__ sums, float* __restrict__ loss, float* __restrict__ dx) {
  const long long total = (long long)B * P;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += (2.f * sums[3 * b] + eps) / (sums[3 * b + 1] + sums[3 * b + 2] + eps);
    loss[0] = 1.f - s / (float)B;
  }
  if (!dx) return;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / P);
    const float I = sums[3 * b], U = sums[3 * b + 1] + sums[3 * b + 2];
    const float p = sigmoid_f(ld(x + i));
    const float tv = ld(t + i);
    // dice = (2I+eps)/(U+eps); d dice/dp = (2t(U+eps) - (2I+eps))/(U+eps)^2
    const float dd = (2.f * tv * (U + eps) - (2.f * I + eps)) / ((U + eps) * (U + eps));
    dx[i] = -dd * p * (1.f - p) / (float)B;
  }
}

// ------------------------------------------------------------ recon
__device__ __forceinline__ void lin_r(int o, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float src = (o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

// lin_r with the scale (float)in / (float)out precomputed (same float, same result)
__device__ __forceinline__ void lin_rs(int o, int in, float scale, int& i0, int& i1, float& l1) {
  float src = (o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

struct ReconArgs {
  const void* r[5];      // recon maps [B][h][w] (single channel, channel stride ldr)
  int ldr[5];
  int target[5];         // 0: target A, 1: target B, 2: (ca*A + cb*B)
  int nterms;
  const float* tA;       // [B][S][S] channel means
  const float* tB;
  float ca, cb;          // combination for target 2
  int B, h, w, S;
  float sc_h, sc_w;      // (float)h / S, (float)w / S
  float* sums;           // [5] loss sums (atomic)
  float* grads[5];       // [B][h][w] fp32 (atomic accumulation, unit-upstream, scaled by 1/(B*S*S))
};

// block per (b, output row y); thread per output column x
template <typename T>
__global__ void k_recon(ReconArgs a) {
  __shared__ float rowacc[5][2][64];  // contributions to input rows (i0, i1) for w <= 64 columns
  __shared__ float red[16];
  const int b = blockIdx.x / a.S, y = blockIdx.x % a.S;
  int i0, i1;
  float ly;
  lin_r(y, a.h, a.S, i0, i1, ly);
  for (int t = threadIdx.x; t < 5 * 2 * 64; t += blockDim.x) (&rowacc[0][0][0])[t] = 0.f;
  __syncthreads();
  const float inv_n = 1.f / ((float)a.B * a.S * a.S);
  float part[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int x = threadIdx.x; x < a.S; x += blockDim.x) {
    int j0, j1;
    float lx;
    lin_r(x, a.w, a.S, j0, j1, lx);
    const size_t tp = ((size_t)b * a.S + y) * a.S + x;
    const float tAv = a.tA ? a.tA[tp] : 0.f, tBv = a.tB ? a.tB[tp] : 0.f;
    for (int k = 0; k < a.nterms; ++k) {
      const T* R = (const T*)a.r[k] + (size_t)b * a.h * a.w * a.ldr[k];
      const int ld_ = a.ldr[k];
      const float v = (1.f - ly) * ((1.f - lx) * ld(R + (i0 * a.w + j0) * ld_) + lx * ld(R + (i0 * a.w + j1) * ld_)) +
                      ly * ((1.f - lx) * ld(R + (i1 * a.w + j0) * ld_) + lx * ld(R + (i1 * a.w + j1) * ld_));
      float tv = a.target[k] == 0 ? tAv : (a.target[k] == 1 ? tBv : a.ca * tAv + a.cb * tBv);
      tv = fminf(fmaxf(tv, 0.f), 1.f);
      const float s = sigmoid_f(v);
      const float p = fminf(fmaxf(s, 0.f), 1.f);
      const float d = p - tv;
      const float q = sqrtf(d * d + 1e-6f);
      part[k] += q;
      // dL/dv = d/q * dsig (clamp is identity on (0,1))
      const float g = d / q * s * (1.f - s) * inv_n;
      atomicAdd(&rowacc[k][0][j0], (1.f - ly) * (1.f - lx) * g);
      atomicAdd(&rowacc[k][0][j1], (1.f - ly) * lx * g);
      atomicAdd(&rowacc[k][1][j0], ly * (1.f - lx) * g);
      atomicAdd(&rowacc[k][1][j1], ly * lx * g);
    }
  }
  __syncthreads();
  for (int k = 0; k < a.nterms; ++k) {
    const float s = block_sum(part[k], red);
    if (threadIdx.x == 0) atomicAdd(a.sums + k, s);
    if (a.grads[k])
      for (int t = threadIdx.x; t < 2 * a.w; t += blockDim.x) {
        const int which = t / a.w, j = t % a.w;
        const float v = rowacc[k][which][j];
        if (v != 0.f) atomicAdd(a.grads[k] + ((size_t)b * a.h + (which ? i1 : i0)) * a.w + j, v);
      }
  }
}

// Band form: block = (b, band of RB output rows). Per output row every
// thread computes the loss term and its gradient g(y, x) for its columns
// into LDS (no atomics); column threads j then gather their bilinear
// window of g (the source column is monotonic in x), and the band's
// contributions to its (<= RB*h/S + 2) input rows are accumulated in LDS
// registers and added to the global gradient with one atomic per element
// per band (<= 3 adders per element). Loss sums: one atomic per term per
// block.
constexpr int RECON_RB = 8;
constexpr int RECON_MAXS = 512;
template <typename T>
__global__ void __launch_bounds__(256) k_recon_band(ReconArgs a) {
  __shared__ float G[5][RECON_MAXS];
  __shared__ float acc[5][RECON_RB + 2][64];
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int y0 = blockIdx.y * RECON_RB, y1 = min(a.S, y0 + RECON_RB);
  const float inv_n = 1.f / ((float)a.B * a.S * a.S);
  int ib0, tmp;
  float ftmp;
  lin_r(y0, a.h, a.S, ib0, tmp, ftmp);  // first input row touched by this band
  for (int t = threadIdx.x; t < 5 * (RECON_RB + 2) * 64; t += blockDim.x) (&acc[0][0][0])[t] = 0.f;
  float part[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int y = y0; y < y1; ++y) {
    int i0, i1;
    float ly;
    lin_r(y, a.h, a.S, i0, i1, ly);
    __syncthreads();  // G reuse
    for (int x = threadIdx.x; x < a.S; x += blockDim.x) {
      int j0, j1;
      float lx;
      lin_r(x, a.w, a.S, j0, j1, lx);
      const size_t tp = ((size_t)b * a.S + y) * a.S + x;
      const float tAv = a.tA ? a.tA[tp] : 0.f, tBv = a.tB ? a.tB[tp] : 0.f;
      for (int k = 0; k < a.nterms; ++k) {
        const T* R = (const T*)a.r[k] + (size_t)b * a.h * a.w * a.ldr[k];
        const int ld_ = a.ldr[k];
        const float v = (1.f - ly) * ((1.f - lx) * ld(R + (i0 * a.w + j0) * ld_) + lx * ld(R + (i0 * a.w + j1) * ld_)) +
                        ly * ((1.f - lx) * ld(R + (i1 * a.w + j0) * ld_) + lx * ld(R + (i1 * a.w + j1) * ld_));
        float tv = a.target[k] == 0 ? tAv : (a.target[k] == 1 ? tBv : a.ca * tAv + a.cb * tBv);
        tv = fminf(fmaxf(tv, 0.f), 1.f);
        const float sg = sigmoid_f(v);
        const float pp = fminf(fmaxf(sg, 0.f), 1.f);
        const float d = pp - tv;
        const float q = sqrtf(d * d + 1e-6f);
        part[k] += q;
        G[k][x] = d / q * sg * (1.f - sg) * inv_n;  // dL/dv (clamp is identity on (0,1))
      }
    }
    __syncthreads();
    // column gather: thread (k, j) sums its window of x
    for (int t = threadIdx.x; t < a.nterms * a.w; t += blockDim.x) {
      const int k = t / a.w, j = t % a.w;
      // x whose source column j0 or j1 is j lie in [xl, xh)
      int xl = (int)floorf(((float)j - 1.f + 0.5f) * a.S / a.w - 0.5f) - 1;
      int xh = (int)ceilf(((float)j + 1.f + 0.5f) * a.S / a.w - 0.5f) + 2;
      xl = max(xl, 0);
      xh = min(xh, a.S);
      float h = 0.f;
      for (int x = xl; x < xh; ++x) {
        int j0, j1;
        float lx;
        lin_r(x, a.w, a.S, j0, j1, lx);
        const float gv = G[k][x];
        if (j0 == j) h += (1.f - lx) * gv;
        if (j1 == j) h += lx * gv;
      }
      if (a.grads[k]) {
        acc[k][i0 - ib0][j] += (1.f - ly) * h;
        acc[k][i1 - ib0][j] += ly * h;
      }
    }
  }
  __syncthreads();
  for (int k = 0; k < a.nterms; ++k) {
    const float sm = block_sum(part[k], red);
    if (threadIdx.x == 0) atomicAdd(a.sums + k, sm);
  }
  int ie, jt;
  float ft;
  lin_r(y1 - 1, a.h, a.S, jt, ie, ft);  // last input row touched
  const int nrows = ie - ib0 + 1;
  for (int t = threadIdx.x; t < a.nterms * nrows * a.w; t += blockDim.x) {
    const int k = t / (nrows * a.w), rem = t % (nrows * a.w), r = rem / a.w, j = rem % a.w;
    const float v = acc[k][r][j];
    if (a.grads[k] && v != 0.f) atomicAdd(a.grads[k] + ((size_t)b * a.h + ib0 + r) * a.w + j, v);
  }
}

// Streaming form (the recon launch of a fusion step at HBM rate), two
// passes, no atomics (deterministic):
//  1. k_recon_stream, block = (b, band of RECON_RB output rows), thread =
//     output column(s). The band's <= 3 source rows of every map are staged
//     in LDS once; each thread x-interpolates them for its column, then per
//     output row needs one FMA for the bilinear value, the loss term and
//     dL/dv (the targets streamed once, coalesced). The gradient contracts
//     separably: over the band's rows in registers (A[k][r][x] = sum_y
//     wy(y, r) g(y, x)), then over x through LDS; the band's <= 3 x w
//     source-row contributions per map and its loss partial sums go to a
//     workspace slab with plain stores.
//  2. k_recon_finish: per (map, b) block, every source element sums the
//     (<= 3) bands covering its row in band order; one more block sums the
//     loss partials in block order. Same-address atomics (the loss sums of
//     1024 blocks onto 5 addresses) serialised the one-pass form.
constexpr int RECON_NR = 3;   // source rows a band may touch
constexpr int RECON_XPT = 2;  // output columns per thread (S <= 512)
template <typename T>
__global__ void __launch_bounds__(256) k_recon_stream(ReconArgs a, float* __restrict__ ws) {
  __shared__ float Rs[5][RECON_NR][64];
  __shared__ float red5[5][4];
  // sized by S at launch (5 * 3 * S + S floats + S shorts): at S = 256 half the static
  // RECON_MAXS footprint, so twice the resident blocks per CU
  extern __shared__ __attribute__((aligned(16))) float rdyn[];
  float* AccF = rdyn;                                     // [5][RECON_NR][S]
  float* Lx = rdyn + 5 * RECON_NR * a.S;                  // column x: bilinear weight of j1
  short* J0 = (short*)(rdyn + 5 * RECON_NR * a.S + a.S);  // column x: source column j0 (j1 = j0 + (j0 < w-1))
#define Acc(k, r, x) AccF[((k) * RECON_NR + (r)) * a.S + (x)]
  const int b = blockIdx.x, q = blockIdx.y, nb = gridDim.y;
  const int y0 = q * RECON_RB, y1 = min(a.S, y0 + RECON_RB);
  const int tid = threadIdx.x;
  const float inv_n = 1.f / ((float)a.B * a.S * a.S);
  // the band's target values of this thread's columns: every HBM load issued first, so their
  // latency overlaps the staging below (one exposed latency per block, not two)
  float tAr[RECON_XPT][RECON_RB], tBr[RECON_XPT][RECON_RB];
#pragma unroll
  for (int u = 0; u < RECON_XPT; ++u) {
    const int x = tid + u * 256;
    const bool xin = x < a.S;
    const float* pA = (a.tA && xin) ? a.tA + ((size_t)b * a.S + y0) * a.S + x : nullptr;
    const float* pB = (a.tB && xin) ? a.tB + ((size_t)b * a.S + y0) * a.S + x : nullptr;
#pragma unroll
    for (int yy = 0; yy < RECON_RB; ++yy) {
      const bool in = y0 + yy < y1;
      tAr[u][yy] = (pA && in) ? __builtin_nontemporal_load(pA + (size_t)yy * a.S) : 0.f;
      tBr[u][yy] = (pB && in) ? __builtin_nontemporal_load(pB + (size_t)yy * a.S) : 0.f;
    }
  }
  int ib0, ie, tmp;
  float ftmp;
  lin_rs(y0, a.h, a.sc_h, ib0, tmp, ftmp);
  lin_rs(y1 - 1, a.h, a.sc_h, tmp, ie, ftmp);
  for (int x = tid; x < a.S; x += blockDim.x) {
    int j0, j1;
    float lx;
    lin_rs(x, a.w, a.sc_w, j0, j1, lx);
    J0[x] = (short)j0;
    Lx[x] = lx;
  }
  const int nrows = ie - ib0 + 1;  // <= RECON_NR (checked by the launcher)
  // the band's source rows: all of a thread's (<= 4) loads in flight before its LDS stores (a
  // load -> store chain per element paid the load latency four times)
  static_assert(5 * RECON_NR * 64 <= 4 * 256, "recon staging: 4 elements per thread");
  float sv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = tid + u * 256;
    const int k = t / (RECON_NR * 64), rem = t - k * (RECON_NR * 64), r = rem / 64, j = rem - r * 64;
    sv[u] = 0.f;
    if (t < 5 * RECON_NR * 64 && k < a.nterms && r < nrows && j < a.w) {
      const T* R = (const T*)a.r[k] + ((size_t)b * a.h * a.w + (size_t)(ib0 + r) * a.w + j) * a.ldr[k];
      sv[u] = ld(R);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = tid + u * 256;
    if (t < 5 * RECON_NR * 64) {
      const int k = t / (RECON_NR * 64), rem = t - k * (RECON_NR * 64), r = rem / 64, j = rem - r * 64;
      Rs[k][r][j] = sv[u];
    }
  }
  __syncthreads();
  float part[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < RECON_XPT; ++u) {
    const int x = tid + u * 256;
    if (x >= a.S) break;
    int j0, j1;
    float lx;
    lin_rs(x, a.w, a.sc_w, j0, j1, lx);
    float rx[5][RECON_NR], A[5][RECON_NR];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int r = 0; r < RECON_NR; ++r) {
        rx[k][r] = (1.f - lx) * Rs[k][r][j0] + lx * Rs[k][r][j1];
        A[k][r] = 0.f;
      }
#pragma unroll
    for (int yy = 0; yy < RECON_RB; ++yy) {
      const int y = y0 + yy;
      if (y >= y1) break;
      int i0, i1;
      float ly;
      lin_rs(y, a.h, a.sc_h, i0, i1, ly);
      const int q0 = i0 - ib0, q1 = i1 - ib0;
      const float tAv = tAr[u][yy], tBv = tBr[u][yy];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        if (k >= a.nterms) break;
        // the x-interpolated source rows q0 / q1 (<= 3 rows: selects, no dynamic register indexing)
        const float r0 = q0 == 0 ? rx[k][0] : (q0 == 1 ? rx[k][1] : rx[k][2]);
        const float r1 = q1 == 0 ? rx[k][0] : (q1 == 1 ? rx[k][1] : rx[k][2]);
        const float v = (1.f - ly) * r0 + ly * r1;
        float tv = a.target[k] == 0 ? tAv : (a.target[k] == 1 ? tBv : a.ca * tAv + a.cb * tBv);
        tv = fminf(fmaxf(tv, 0.f), 1.f);
        const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-v));
        const float pp = fminf(fmaxf(sg, 0.f), 1.f);
        const float d = pp - tv;
        const float e2 = d * d + 1e-6f;
        const float rq = __builtin_amdgcn_rsqf(e2);  // 1 / sqrt(d^2 + eps): the term is e2 * rq, d/term = d * rq
        part[k] += e2 * rq;
        const float g = d * rq * sg * (1.f - sg) * inv_n;  // dL/dv (the clamp is the identity on (0,1))
        const float g0 = (1.f - ly) * g, g1 = ly * g;
#pragma unroll
        for (int r = 0; r < RECON_NR; ++r) A[k][r] += (q0 == r ? g0 : 0.f) + (q1 == r ? g1 : 0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int r = 0; r < RECON_NR; ++r) Acc(k, r, x) = A[k][r];
  }
  __syncthreads();
  // x-contraction: (k, r, j) sums the columns x whose source column j0 or j1 is j -> slab row r of band q
  float* G = ws + (size_t)a.B * nb * 5;
  for (int t = tid; t < a.nterms * RECON_NR * a.w; t += blockDim.x) {
    const int k = t / (RECON_NR * a.w), rem = t - k * (RECON_NR * a.w), r = rem / a.w, j = rem - r * a.w;
    float h = 0.f;
    if (r < nrows && a.grads[k]) {
      int xl = (int)floorf(((float)j - 1.f + 0.5f) * a.S / a.w - 0.5f) - 1;
      int xh = (int)ceilf(((float)j + 1.f + 0.5f) * a.S / a.w - 0.5f) + 2;
      xl = max(xl, 0);
      xh = min(xh, a.S);
      for (int x = xl; x < xh; ++x) {
        const int j0 = J0[x], j1 = j0 + (j0 < a.w - 1 ? 1 : 0);
        const float lx = Lx[x], av = Acc(k, r, x);
        if (j0 == j) h += (1.f - lx) * av;
        if (j1 == j) h += lx * av;
      }
    }
    G[(((size_t)k * a.B + b) * nb + q) * RECON_NR * a.w + r * a.w + j] = h;
  }
  // the five loss partials in one block reduction (one barrier)
#pragma unroll
  for (int k = 0; k < 5; ++k) part[k] = wave_sum(part[k]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < 5; ++k) red5[k][tid >> 6] = part[k];
  __syncthreads();
  if (tid < a.nterms) {
    float sm = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) sm += red5[tid][i];
    ws[((size_t)b * nb + q) * 5 + tid] = sm;
  }
}

#undef Acc

// pass 2: one thread per gradient element (map k, item b, source row i,
// column j) sums the (<= 3) band slabs covering row i, in band order; the
// last block sums the loss partials in block order (fixed orders:
// deterministic)
__global__ void __launch_bounds__(256) k_recon_finish(ReconArgs a, const float* __restrict__ ws, int nb) {
  const int tid = threadIdx.x;
  const long long per = (long long)a.B * a.h * a.w;
  if ((int)blockIdx.x == (int)gridDim.x - 1) {
    __shared__ float red[16];
    const int nblk = a.B * nb;
    for (int k = 0; k < a.nterms; ++k) {
      float s = 0.f;
      for (int i = tid; i < nblk; i += blockDim.x) s += ws[(size_t)i * 5 + k];
      s = block_sum(s, red);
      if (tid == 0) a.sums[k] = s;
    }
    return;
  }
  const long long t = (long long)blockIdx.x * blockDim.x + tid;
  if (t >= per * a.nterms) return;
  const int k = (int)(t / per);
  const long long r = t - (long long)k * per;
  const int b = (int)(r / (a.h * a.w)), e = (int)(r - (long long)b * a.h * a.w);
  if (!a.grads[k]) return;
  const int i = e / a.w, j = e - (e / a.w) * a.w;
  const float* G = ws + (size_t)a.B * nb * 5 + ((size_t)k * a.B + b) * nb * RECON_NR * a.w;
  // bands whose source rows [ib0, ie] contain i: around the band of output row (i + 0.5) * S / h
  const int qc = (int)(((float)i + 0.5f) * a.S / a.h) / RECON_RB;
  float s = 0.f;
  for (int q = max(0, qc - 2); q <= min(nb - 1, qc + 2); ++q) {
    int ib0, ie, tmp;
    float ftmp;
    lin_rs(q * RECON_RB, a.h, a.sc_h, ib0, tmp, ftmp);
    lin_rs(min(a.S, q * RECON_RB + RECON_RB) - 1, a.h, a.sc_h, tmp, ie, ftmp);
    if (i >= ib0 && i <= ie) s += G[(size_t)q * RECON_NR * a.w + (i - ib0) * a.w + j];
  }
  a.grads[k][(size_t)b * a.h * a.w + e] = s;
}

// ------------------------------------------------------------ mimic
// pair i: student S_i = s + i*sstride, teacher T_i = t + i*tstride, each an
// [HW][C] NHWC map (channel stride ld). mimic_feat_loss flattens [C,H,W] to
// [C, HW]: per-channel cosine over HW; loss = mean over channels and pairs.
// Gradient only for the student (teacher detached).
template <typename T>
__global__ void k_mimic(const T* __restrict__ sbase, const T* __restrict__ tbase, long long sstride,
                        long long tstride, int ldm, int HW, int C, int npairs, float eps_norm, float eps_clamp,
                        float* __restrict__ part, T* __restrict__ dstudent, long long dstride) {
  // block per (pair, channel)
  __shared__ float red[16];
  const int pr = blockIdx.x / C, c = blockIdx.x % C;
  const T* S = sbase + (size_t)pr * sstride + c;
  const T* Tt = tbase + (size_t)pr * tstride + c;
  float ss = 0.f, tt = 0.f, st_ = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    const float sv = ld(S + (size_t)p * ldm), tv = ld(Tt + (size_t)p * ldm);
    ss += sv * sv;
    tt += tv * tv;
    st_ += sv * tv;
  }
  ss = block_sum(ss, red);
  tt = block_sum(tt, red);
  st_ = block_sum(st_, red);
  const float ns = fmaxf(sqrtf(ss), eps_norm), nt = fmaxf(sqrtf(tt), eps_norm);
  const float cos = st_ / (ns * nt);
  const float lo = -1.f + eps_clamp, hi = 1.f - eps_clamp;
  if (threadIdx.x == 0) part[blockIdx.x] = (1.f - fminf(fmaxf(cos, lo), hi)) / (float)(C * npairs);
  if (dstudent) {
    const bool pass = cos >= lo && cos <= hi;
    const float scale = -1.f / (float)(C * npairs);
    const bool snorm_active = sqrtf(ss) > eps_norm;
    T* D = dstudent + (size_t)pr * dstride + c;
    for (int p = threadIdx.x; p < HW; p += blockDim.x) {
      float g = 0.f;
      if (pass) {
        const float sv = ld(S + (size_t)p * ldm), tv = ld(Tt + (size_t)p * ldm);
        g = tv / (ns * nt) - (snorm_active ? cos * sv / (ns * ns) : 0.f);
        g *= scale;
      }
      st(D + (size_t)p * ldm, g);
    }
  }
}

__global__ void k_scale_by(const float* __restrict__ src, long long n, const float* __restrict__ s, float mul,
                           float* __restrict__ dst) {
  const float k = s[0] * mul;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = src[i] * k;
}

template <typename T>
__global__ void k_scale_by_cast(const float* __restrict__ src, long long n, const float* __restrict__ s, float mul,
                                T* __restrict__ dst, int ldd, int C) {
  const float k = s[0] * mul;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / C;
    const int c = (int)(i - m * C);
    st(dst + m * ldd + c, src[i] * k);
  }
}

static inline int gsz(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}


// ------------------------------------------------ loss assembly of one step
// total = sum_i coef_i * v_i * (w if flagged) over the scalar criterion values of
// _shared_step (train_fusion.py:246-300: cls + lambda_mask * mean of the three
// mask losses + aux_w * (lambda_recon * recon + lambda_mimic * mimic)), plus the
// reported group sums (mask / recon / mimic values), in one launch; the
// backward writes every term's gradient in one more (was ~40 scalar aten
// launches forward + backward).
struct LossPlan {
  const float* p[DMF_LOSS_MAX];
  float coef[DMF_LOSS_MAX];
  float gcoef[DMF_LOSS_MAX];
  int flags[DMF_LOSS_MAX];  // bit 0: times w; bits 1..: group + 1 (0 = none)
  int n, ng;
};

__global__ void k_loss_combine(LossPlan pl, const float* __restrict__ w, float* __restrict__ total_out,
                               float* __restrict__ groups) {
  if (threadIdx.x != 0) return;
  const float wv = w ? *w : 1.f;
  float total = 0.f, g[DMF_LOSS_MAX];
  for (int k = 0; k < pl.ng; ++k) g[k] = 0.f;
  for (int i = 0; i < pl.n; ++i) {
    const float v = *pl.p[i];
    total += pl.coef[i] * v * ((pl.flags[i] & 1) ? wv : 1.f);
    const int grp = (pl.flags[i] >> 1) - 1;
    if (grp >= 0 && grp < pl.ng) g[grp] += pl.gcoef[i] * v;
  }
  total_out[0] = total;
  for (int k = 0; k < pl.ng; ++k) groups[k] = g[k];
}

__global__ void k_loss_combine_bwd(LossPlan pl, const float* __restrict__ w, const float* __restrict__ dtotal,
                                   float* __restrict__ grads) {
  const int i = threadIdx.x;
  if (i >= pl.n) return;
  const float wv = w ? *w : 1.f;
  grads[i] = *dtotal * pl.coef[i] * ((pl.flags[i] & 1) ? wv : 1.f);
}

// torch.argmax(logits, 1) == labels, averaged (train_fusion.py:302-303): first maximum, NaN
// counts as the maximum (torch's rule)
__global__ void k_batch_accuracy(const float* __restrict__ z, const long long* __restrict__ labels, int B, int K,
                                 float* __restrict__ out) {
  __shared__ float red[16];
  float hit = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float* r = z + (size_t)b * K;
    int best = 0;
    float bv = r[0];
    for (int k = 1; k < K; ++k) {
      const float v = r[k];
      if (!(bv != bv) && ((v != v) || v > bv)) {
        bv = v;
        best = k;
      }
    }
    hit += best == labels[b] ? 1.f : 0.f;
  }
  hit = block_sum(hit, red);
  if (threadIdx.x == 0) out[0] = hit / (float)B;
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_focal_loss(const float* logits, const long long* labels, const float* soft_targets, int B, int K,
                              float smoothing, int use_smoothing, const float* class_weights, float gamma,
                              int reduction, float* loss, float* per_row, float* dlogits, void* stream) {
  DMF_CHECK_ARG(logits && (labels || soft_targets) && B > 0 && K > 1 && K <= 64 && reduction >= 0 && reduction <= 2,
                "dmf_focal_loss: bad args (K=%d, reduction=%d)", K, reduction);
  hipLaunchKernelGGL(k_focal, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, labels, soft_targets, B, K,
                     smoothing, use_smoothing, class_weights, gamma, reduction, loss, per_row, dlogits);
  DMF_LAUNCH_CHECK("dmf_focal_loss");
  return 0;
}

extern "C" int dmf_label_smooth(const long long* labels, int B, int K, float smoothing, float* out, void* stream) {
  DMF_CHECK_ARG(labels && out && B > 0 && K > 1, "dmf_label_smooth: bad args");
  hipLaunchKernelGGL(k_label_smooth, dim3(cdiv(B * K, 256)), dim3(256), 0, (hipStream_t)stream, labels, B, K,
                     smoothing, out);
  DMF_LAUNCH_CHECK("dmf_label_smooth");
  return 0;
}

extern "C" int dmf_soft_dice(int dtype, const void* logits, const float* target, int B, int P, float eps,
                             float* sums_ws, float* loss, float* dlogits, void* stream) {
  DMF_CHECK_ARG(logits && target && sums_ws && loss && B > 0 && P > 0, "dmf_soft_dice: bad args");
  hipStream_t s = (hipStream_t)stream;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_dice_sums<T, float>), dim3(B), dim3(256), 0, s, (const T*)logits, target, P,
                       sums_ws);
    hipLaunchKernelGGL((k_dice_grad<T, float>), dim3(gsz((long long)B * P)), dim3(256), 0, s,
                       (const T*)logits, target, B, P, eps, sums_ws, loss, dlogits));
  DMF_LAUNCH_CHECK("dmf_soft_dice");
  return 0;
}

// recon terms: up to 5 maps r_k ([B][h][w], channel stride ldr_k) against target sel_k in {0:A,1:B,2:ca*A+cb*B}.
// sums[k] += sum of charbonnier terms (caller divides by B*S*S); grads[k] += unit-upstream grads (scaled 1/(B*S*S)).
// floats of the two-pass streaming form's workspace, 0 where it does not apply (the caller then passes
// ws = nullptr and zeroed sums / gradients for the atomic one-pass forms)
extern "C" int dmf_recon_ws_floats(int nterms, int B, int h, int w, int S) {
  // source rows a band of RECON_RB output rows touches: ceil(RB*h/S) + 1 (+1 clamp slack) <= RECON_NR
  const bool ok = nterms >= 1 && nterms <= 5 && B > 0 && S <= RECON_MAXS && S <= 256 * RECON_XPT && h <= S &&
                  w <= 64 && (RECON_RB * h + S - 1) / S + 2 <= RECON_NR;
  if (!ok) return 0;
  const long long nb = cdiv(S, RECON_RB);
  const long long n = (long long)B * nb * 5 + (long long)nterms * B * nb * RECON_NR * w;
  return n < (1LL << 30) ? (int)n : 0;
}

extern "C" int dmf_recon_loss(int dtype, int nterms, const void* r0, const void* r1, const void* r2, const void* r3,
                              const void* r4, int ldr0, int ldr1, int ldr2, int ldr3, int ldr4, int sel0, int sel1,
                              int sel2, int sel3, int sel4, const float* tA, const float* tB, float ca, float cb,
                              int B, int h, int w, int S, float* sums, float* g0, float* g1, float* g2, float* g3,
                              float* g4, float* ws, void* stream) {
  DMF_CHECK_ARG(nterms >= 1 && nterms <= 5 && sums && w <= 64 && B > 0 && S > 0, "dmf_recon_loss: bad args");
  ReconArgs a{};
  const void* rs[5] = {r0, r1, r2, r3, r4};
  const int lds[5] = {ldr0, ldr1, ldr2, ldr3, ldr4};
  const int sels[5] = {sel0, sel1, sel2, sel3, sel4};
  float* gs[5] = {g0, g1, g2, g3, g4};
  for (int k = 0; k < 5; ++k) {
    a.r[k] = rs[k];
    a.ldr[k] = lds[k];
    a.target[k] = sels[k];
    a.grads[k] = gs[k];
    if (k < nterms) DMF_CHECK_ARG(rs[k] != nullptr, "dmf_recon_loss: missing map %d", k);
  }
  a.nterms = nterms;
  a.tA = tA; a.tB = tB; a.ca = ca; a.cb = cb;
  a.B = B; a.h = h; a.w = w; a.S = S;
  a.sc_h = (float)h / (float)S;
  a.sc_w = (float)w / (float)S;
  a.sums = sums;
  if (ws != nullptr) {
    // two-pass streaming form: sums and gradients are WRITTEN (no zeroing needed)
    DMF_CHECK_ARG(dmf_recon_ws_floats(nterms, B, h, w, S) > 0, "dmf_recon_loss: workspace given for a shape "
                  "outside the streaming form (B=%d h=%d w=%d S=%d)", B, h, w, S);
    const int nb = cdiv(S, RECON_RB);
    const dim3 g(B, nb);
    const size_t lds = (size_t)(5 * RECON_NR * S + S) * sizeof(float) + (size_t)S * sizeof(short);
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_recon_stream<T>, g, dim3(256), lds, (hipStream_t)stream, a, ws));
    hipLaunchKernelGGL(k_recon_finish, dim3(cdiv((long long)nterms * B * h * w, 256) + 1), dim3(256), 0,
                       (hipStream_t)stream, a, ws, nb);
  } else if (S <= RECON_MAXS && h <= S && (RECON_RB * h + S - 1) / S + 2 <= RECON_RB + 2) {
    const dim3 g(B, cdiv(S, RECON_RB));
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_recon_band<T>, g, dim3(256), 0, (hipStream_t)stream, a));
  } else DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_recon<T>, dim3(B * S), dim3(256), 0, (hipStream_t)stream, a));
  DMF_LAUNCH_CHECK("dmf_recon_loss");
  return 0;
}

extern "C" int dmf_mimic_loss(int dtype, const void* student, const void* teacher, long long sstride,
                              long long tstride, int ld, int HW, int C, int npairs, float* loss, void* dstudent,
                              long long dstride, float* ws, void* stream) {
  DMF_CHECK_ARG(student && teacher && loss && ws && npairs >= 1 && C > 0 && HW > 0, "dmf_mimic_loss: bad args");
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mimic<T>, dim3(npairs * C), dim3(256), 0, (hipStream_t)stream, (const T*)student,
                       (const T*)teacher, sstride, tstride, ld, HW, C, npairs, 1e-12f, 1e-6f, ws,
                       (T*)dstudent, dstride));
  DMF_LAUNCH_CHECK("dmf_mimic_loss");
  return dmf_colsum_f32(ws, 1, npairs * C, 1, loss, 1, stream);  // the terms in (pair, channel) order
}

extern "C" int dmf_scale_by(const float* src, long long n, const float* scalar, float mul, float* dst, void* stream) {
  DMF_CHECK_ARG(src && scalar && dst, "dmf_scale_by: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_scale_by, dim3(gsz(n)), dim3(256), 0, (hipStream_t)stream, src, n, scalar, mul, dst);
  DMF_LAUNCH_CHECK("dmf_scale_by");
  return 0;
}

extern "C" int dmf_scale_by_cast(int dtype, const float* src, long long M, int C, const float* scalar, float mul,
                                 void* dst, int ldd, void* stream) {
  DMF_CHECK_ARG(src && scalar && dst, "dmf_scale_by_cast: bad args");
  const long long n = M * C;
  if (n == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_scale_by_cast<T>, dim3(gsz(n)), dim3(256), 0, (hipStream_t)stream, src, n, scalar, mul,
                       (T*)dst, ldd, C));
  DMF_LAUNCH_CHECK("dmf_scale_by_cast");
  return 0;
}

static int loss_plan(int n, const unsigned long long* ptrs, const float* coef, const int* flags, const float* gcoef,
                     int ng, LossPlan& pl) {
  if (n < 1 || n > DMF_LOSS_MAX || ng < 0 || ng > DMF_LOSS_MAX || !ptrs || !coef || !flags) return -1;
  pl.n = n;
  pl.ng = ng;
  for (int i = 0; i < n; ++i) {
    pl.p[i] = (const float*)(uintptr_t)ptrs[i];
    pl.coef[i] = coef[i];
    pl.gcoef[i] = gcoef ? gcoef[i] : 0.f;
    pl.flags[i] = flags[i];
    if (!pl.p[i]) return -1;
  }
  return 0;
}

extern "C" int dmf_loss_combine(int n, const unsigned long long* ptrs, const float* coef, const int* flags,
                                const float* gcoef, int ngroups, const float* w, float* total, float* groups,
                                void* stream) {
  LossPlan pl;
  DMF_CHECK_ARG(total && (groups || ngroups == 0) && loss_plan(n, ptrs, coef, flags, gcoef, ngroups, pl) == 0,
                "dmf_loss_combine: bad args");
  hipLaunchKernelGGL(k_loss_combine, dim3(1), dim3(64), 0, (hipStream_t)stream, pl, w, total, groups);
  DMF_LAUNCH_CHECK("dmf_loss_combine");
  return 0;
}

extern "C" int dmf_loss_combine_bwd(int n, const float* coef, const int* flags, const float* w, const float* dtotal,
                                    float* grads, void* stream) {
  LossPlan pl;
  unsigned long long dummy[DMF_LOSS_MAX];
  for (int i = 0; i < DMF_LOSS_MAX; ++i) dummy[i] = 1;
  DMF_CHECK_ARG(dtotal && grads && loss_plan(n, dummy, coef, flags, nullptr, 0, pl) == 0,
                "dmf_loss_combine_bwd: bad args");
  hipLaunchKernelGGL(k_loss_combine_bwd, dim3(1), dim3(64), 0, (hipStream_t)stream, pl, w, dtotal, grads);
  DMF_LAUNCH_CHECK("dmf_loss_combine_bwd");
  return 0;
}

extern "C" int dmf_batch_accuracy(const float* logits, const long long* labels, int B, int K, float* out,
                                  void* stream) {
  DMF_CHECK_ARG(logits && labels && out && B > 0 && K > 0, "dmf_batch_accuracy: bad args");
  hipLaunchKernelGGL(k_batch_accuracy, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, labels, B, K, out);
  DMF_LAUNCH_CHECK("dmf_batch_accuracy");
  return 0;
}
