// oaz_train.hip — the training step on gfx950: gather a batch from the
// replay buffer, ConvResNet::forward(train=true) (net.rs:215-232, BN on batch statistics),
// alphaloss (net.rs:234-243), backward, and tch's SGD (train.rs:181-186, 309).
//
// Layout. Activations are square-major rows: row = sq * B + b (sq = board square, b = sample),
// 64 fp32 channels per row (the first layer's 21 input planes padded to 32). A 3x3 conv over
// 16 rows of one square reads, for each on-board tap, the 16 contiguous rows of the neighbour
// square, so off-board taps are skipped outright (169 of 225 (square, tap) pairs do work).
//
// Kernels per step (N residual blocks, L = 1 + 2N convs):
//   gather                      samples[idx] -> X0 [R][32], pi [B][50], z [B]
//   per conv: conv_fwd (MFMA 16x16x4 f32, + per-16-row BN partial sums) -> bn_act_cfin (every
//          workgroup finalises the batch statistics from the partials, then applies BN + skip + ReLU)
//   heads: head_conv (1x1, 3 channels) -> bn_fwd_fin x2 -> head_sample (value MLP, policy
//          linear + softmax, loss, their backward, per-sample) -> head_bwd_fin -> head_bwd_rows
//   per conv, last to first: bn_bwd_fin -> bn_bwd_apply -> wgrad (MFMA, per (tap, square)
//          partials) -> wgrad_reduce -> conv_dgrad (the same conv kernel on flipped/transposed
//          weights, epilogue = skip add + ReLU mask + BN-backward partial sums of the layer below)
//   sgd (+ repack of the conv weights for the next step)
// All reductions are two-stage with fixed order (deterministic; no float atomics).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/onitama_az.h"
#include "oaz_device.h"
#include "oaz_host.h"

using namespace oaz;

namespace tr {

constexpr int kC = 64;       // hidden channels
constexpr int kIn = 21;      // input planes
constexpr int kInPad = 32;   // padded input row stride
constexpr int kMaxConv = 1 + 2 * 16;
constexpr int kHeadW = 64 * 25 + 64 + 64 + 1 + 2500 + 50;  // value MLP + policy linear grads
constexpr int kHeadVW = 64 * 25 + 64 + 64 + 1;              // vh_linear1 w,b + vh_linear2 w,b
constexpr int kHConvW = 64 + 1 + 128 + 2;                   // vh_conv w,b + policy_conv w,b

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int nbr(int sq, int t) {
    const int y = sq / 5 + t / 3 - 1, x = sq % 5 + t % 3 - 1;
    return (y >= 0 && y < 5 && x >= 0 && x < 5) ? y * 5 + x : -1;
}

__device__ __forceinline__ float wave_sum16(float v) {  // sum over the 4 lane groups (lane>>4)
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

__device__ __forceinline__ float wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---- gather: create_tensor_from_state (common.rs:26-80) for samples[idx[b]] ----------------------
// threads [0, R): one input row (square, sample); [R, R + 50B): pi; [R + 50B, R + 51B): z
// bi: the batch number, or -1: the one kept on the device (*cur, advanced by the graph replay)
__global__ void k_gather(const oaz_sample* samples, const int32_t* idx_all, const int32_t* cur, int bi, int B,
                         float* X0, float* pi, float* z) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int R = B * 25;
    const int32_t* idx = idx_all + (size_t)(bi >= 0 ? bi : *cur) * B;
    if (t >= R) {
        const int u = t - R;
        if (u < B * 50) pi[u] = samples[idx[u / 50]].pi[u % 50];
        else if (u < B * 51) z[u - B * 50] = samples[idx[u - B * 50]].z;
        return;
    }
    const int b = t % B, sq = t / B;
    const oaz_state st = samples[idx[b]].state;
    const int color = st.to_move & 1;
    const uint32_t bit = sq_bit(sq);
    float* row = X0 + (size_t)(sq * B + b) * kInPad;
    float v[kInPad];
#pragma unroll
    for (int c = 0; c < kInPad; ++c) v[c] = 0.0f;
    v[0] = (st.pawns[0] & bit) ? 1.0f : 0.0f;
    v[1] = (st.kings[0] & bit) ? 1.0f : 0.0f;
    v[2] = (st.pawns[1] & bit) ? 1.0f : 0.0f;
    v[3] = (st.kings[1] & bit) ? 1.0f : 0.0f;
    const int c0 = st.cards[color ? 2 : 0] & 15, c1 = st.cards[color ? 3 : 1] & 15;
#pragma unroll
    for (int c = 0; c < 16; ++c) v[4 + c] = (c == c0 || c == c1) ? 1.0f : 0.0f;
    v[20] = color == OAZ_BLUE ? 1.0f : 0.0f;
#pragma unroll
    for (int c = 0; c < kInPad; c += 4) *reinterpret_cast<float4*>(row + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
}

__global__ void k_set_batch(int32_t* cur, int v, int add) {
    if (threadIdx.x == 0) *cur = add ? *cur + v : v;
}

// ---- 3x3 conv (forward, and dgrad on flipped weights) ------------------------------------------
enum { CONV_FWD = 0, CONV_DGRAD = 1 };

struct ConvArgs {
    const float* in;      // [R][16*chunks]
    const float4* w;      // packed [9][chunks][4 nt][64 lanes]
    const float* bias;    // FWD
    float* out;           // FWD: Z ; DGRAD: m = (dgrad + skip) * (act > 0)
    float* part;          // [nwg][2][64]: FWD sum, sumsq ; DGRAD sum m, sum m*xhat
    const float* act;     // DGRAD: activation of the layer below (ReLU output)
    const float* zprev;   // DGRAD: its pre-BN conv output
    const float* mean;    // DGRAD: its BN batch mean / invstd
    const float* invstd;
    const float* skip;    // DGRAD: residual gradient to add (or null)
    int chunks;           // input channels / 16
    int B;
};

// Workgroup = 64 rows (4 sample tiles of 16, one per wave) of one square x all 64 output
// channels. Per on-board tap the tap's packed weights (CH x 4 n-tiles x 64 lanes float4 = 16 KB
// for 64 input channels) are staged once in LDS (double-buffered) and shared by the 4 waves;
// each wave keeps 4 accumulators (one per 16-channel n-tile), so an A fragment feeds 4 MFMAs.
template <int MODE, int CH, int RG>  // CH = input channels / 16; RG = 16-row groups per workgroup
__global__ __launch_bounds__(256) void k_conv(ConvArgs a) {
    constexpr int NPW = RG;  // n-tiles per wave: 4 waves = RG row groups x (4 / RG) channel splits
    __shared__ float4 sw[2][CH * 256];
    __shared__ float red[RG][2][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, kq = lane >> 4;
    const int rg = wave % RG, n0 = (wave / RG) * NPW;
    const int sq = blockIdx.y, B = a.B, b0 = blockIdx.x * 16 * RG + rg * 16;
    const bool active = b0 < B;  // B is a multiple of 16
    constexpr int rs = 16 * CH;
    f32x4 acc[NPW];
#pragma unroll
    for (int n = 0; n < NPW; ++n) acc[n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // Software pipeline over the on-board taps: the next tap's weights and A fragments are loaded
    // into registers while the current tap's MFMAs run; weights go through a double-buffered LDS.
    // Inactive waves (sample tile past B) load the first tile and discard their results, so the
    // loads and MFMAs stay unconditional and the prefetch registers stay in VGPRs.
    const int bl = active ? b0 : 0;
    float4 wr[CH], av[CH], an[CH];
    // DGRAD: the epilogue's operands (skip, the activation and pre-BN output of the layer below) do not
    // depend on the MFMAs: requested now, they arrive while the taps run instead of after the last one
    float ep[MODE == CONV_DGRAD ? NPW : 1][3][4];
    if constexpr (MODE == CONV_DGRAD) {
#pragma unroll
        for (int n = 0; n < NPW; ++n) {
            const int co = (n0 + n) * 16 + i;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const size_t o = (size_t)(sq * B + bl + kq * 4 + r) * kC + co;
                ep[n][0][r] = a.skip ? a.skip[o] : 0.0f;
                ep[n][1][r] = a.act[o];
                ep[n][2][r] = a.zprev[o];
            }
        }
    }
    int t = 0;
    while (nbr(sq, t) < 0) ++t;
    {
        const float4* wt = a.w + (size_t)t * CH * 256;
#pragma unroll
        for (int k = 0; k < CH; ++k) sw[0][k * 256 + tid] = wt[k * 256 + tid];
        const float* base = a.in + (size_t)(nbr(sq, t) * B + bl + i) * rs + 4 * kq;
#pragma unroll
        for (int g = 0; g < CH; ++g) av[g] = *reinterpret_cast<const float4*>(base + 16 * g);
    }
    __syncthreads();
    for (int cur = 0; t < 9; cur ^= 1) {
        int tn = t + 1;
        while (tn < 9 && nbr(sq, tn) < 0) ++tn;
        const int tl = tn < 9 ? tn : t;  // after the last tap: a harmless reload
        {
            const float4* wt = a.w + (size_t)tl * CH * 256;
#pragma unroll
            for (int k = 0; k < CH; ++k) wr[k] = wt[k * 256 + tid];
            const float* base = a.in + (size_t)(nbr(sq, tl) * B + bl + i) * rs + 4 * kq;
#pragma unroll
            for (int g = 0; g < CH; ++g) an[g] = *reinterpret_cast<const float4*>(base + 16 * g);
        }
#pragma unroll
        for (int g = 0; g < CH; ++g)
#pragma unroll
            for (int n = 0; n < NPW; ++n) {
                const float4 bv = sw[cur][(g * 4 + n0 + n) * 64 + lane];
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g].x, bv.x, acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g].y, bv.y, acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g].z, bv.z, acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g].w, bv.w, acc[n], 0, 0, 0);
            }
#pragma unroll
        for (int k = 0; k < CH; ++k) sw[cur ^ 1][k * 256 + tid] = wr[k];
#pragma unroll
        for (int g = 0; g < CH; ++g) av[g] = an[g];
        __syncthreads();
        t = tn;
    }
    // C/D layout: reg r of lane l = (row 4*(l>>4) + r, col l&15)
#pragma unroll
    for (int n = 0; n < NPW; ++n) {
        const int co = (n0 + n) * 16 + i;
        float s1 = 0.0f, s2 = 0.0f;
        if (active) {
            if (MODE == CONV_FWD) {
                const float bb = a.bias[co];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const size_t o = (size_t)(sq * B + b0 + kq * 4 + r) * kC + co;
                    const float v = acc[n][r] + bb;
                    a.out[o] = v;
                    s1 += v;
                    s2 += v * v;
                }
            } else {
                const float mu = a.mean[co], is = a.invstd[co];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const size_t o = (size_t)(sq * B + b0 + kq * 4 + r) * kC + co;
                    float d = acc[n][r];
                    if (a.skip) d += ep[n][0][r];
                    const float m = ep[n][1][r] > 0.0f ? d : 0.0f;
                    a.out[o] = m;
                    s1 += m;
                    s2 += m * ((ep[n][2][r] - mu) * is);
                }
            }
        }
        s1 = wave_sum16(s1);
        s2 = wave_sum16(s2);
        if (kq == 0) {
            red[rg][0][co] = s1;
            red[rg][1][co] = s2;
        }
    }
    __syncthreads();
    if (tid < 128) {
        const int k = tid >> 6, c = tid & 63;
        const size_t wg = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
        float v = 0.0f;
#pragma unroll
        for (int r = 0; r < RG; ++r) v += red[r][k][c];
        a.part[wg * 128 + tid] = v;
    }
}

// ---- BN finalisation (forward): batch mean / biased var, running stats update ----------------------
// part [nwg][2][pstride] (sum, sumsq) columns coff..coff+C-1; torch batch_norm(training=True):
// y = (x - mean) * invstd * gamma + beta, invstd = 1/sqrt(var_biased + eps);
// running = (1 - m) * running + m * {mean, var_unbiased}.
// Channels c >= split take their running statistics from rmean2 / rvar2 [c - split] (the two heads' BN
// layers in one launch: the value head's channel, then the policy head's two); split = C: one layer.
__global__ __launch_bounds__(1024) void k_bn_fwd_fin(const float* part, int nwg, int pstride, int coff, int C, double N,
                             float* rmean, float* rvar, float bn_mom, float eps, float* mean, float* invstd,
                             int split, float* rmean2, float* rvar2) {
    __shared__ double sh[2][16][64];
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
        double a1[4] = {0.0, 0.0, 0.0, 0.0}, a2[4] = {0.0, 0.0, 0.0, 0.0};
        int w = q;
        for (; w + 48 < nwg; w += 64) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a1[u] += part[(size_t)(w + 16 * u) * 2 * pstride + coff + c];
                a2[u] += part[(size_t)(w + 16 * u) * 2 * pstride + pstride + coff + c];
            }
        }
        for (; w < nwg; w += 16) {
            a1[0] += part[(size_t)w * 2 * pstride + coff + c];
            a2[0] += part[(size_t)w * 2 * pstride + pstride + coff + c];
        }
        s1 = (a1[0] + a1[1]) + (a1[2] + a1[3]);
        s2 = (a2[0] + a2[1]) + (a2[2] + a2[3]);
    }
    sh[0][q][c] = s1;
    sh[1][q][c] = s2;
    __syncthreads();
    if (q == 0 && c < C) {
        s1 = 0.0;
        s2 = 0.0;
        for (int k = 0; k < 16; ++k) {
            s1 += sh[0][k][c];
            s2 += sh[1][k][c];
        }
        const double mu = s1 / N;
        double var = s2 / N - mu * mu;
        if (var < 0.0) var = 0.0;
        mean[c] = (float)mu;
        invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
        float* rm = c < split ? rmean + c : rmean2 + (c - split);
        float* rv = c < split ? rvar + c : rvar2 + (c - split);
        *rm = (float)((1.0 - bn_mom) * *rm + bn_mom * mu);
        *rv = (float)((1.0 - bn_mom) * *rv + bn_mom * var * N / (N - 1.0));
    }
}

// A = relu((Z - mean) * invstd * gamma + beta [+ skip])
__global__ void k_bn_act(const float* Z, const float* mean, const float* invstd, const float* gamma,
                         const float* beta, const float* skip, float* A, long long n) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t * 4 >= n) return;
    const int c = (int)((t * 4) & 63);
    const float4 z = reinterpret_cast<const float4*>(Z)[t];
    float v[4] = {z.x, z.y, z.z, z.w};
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (skip) s = reinterpret_cast<const float4*>(skip)[t];
    const float sk[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float y = (v[k] - mean[c + k]) * invstd[c + k] * gamma[c + k] + beta[c + k];
        if (skip) y += sk[k];
        v[k] = y > 0.0f ? y : 0.0f;
    }
    reinterpret_cast<float4*>(A)[t] = make_float4(v[0], v[1], v[2], v[3]);
}

// Consumer-side forward finalisation: k_bn_fwd_fin and k_bn_act in one launch (0.805 -> 0.762 ms per
// batch-512 step). Every workgroup re-reduces the conv's [nwg][2][64] partials in its prologue (the same fixed
// order in every workgroup, so all of them apply the same statistics); workgroup 0 also writes the batch
// mean / invstd for the backward pass and updates the running statistics.
__global__ __launch_bounds__(1024) void k_bn_act_cfin(const float* part, int nwg, double N, float* rmean, float* rvar,
                                                      float bn_mom, float eps, float* mean_out, float* invstd_out,
                                                      const float* Z, const float* gamma, const float* beta,
                                                      const float* skip, float* A, long long n) {
    __shared__ double sh[2][16][64];
    __shared__ float cf[4][64];  // mean, invstd, gamma, beta
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    {
        double a1[4] = {0.0, 0.0, 0.0, 0.0}, a2[4] = {0.0, 0.0, 0.0, 0.0};
        int w = q;
        for (; w + 48 < nwg; w += 64) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a1[u] += part[(size_t)(w + 16 * u) * 128 + c];
                a2[u] += part[(size_t)(w + 16 * u) * 128 + 64 + c];
            }
        }
        for (; w < nwg; w += 16) {
            a1[0] += part[(size_t)w * 128 + c];
            a2[0] += part[(size_t)w * 128 + 64 + c];
        }
        sh[0][q][c] = (a1[0] + a1[1]) + (a1[2] + a1[3]);
        sh[1][q][c] = (a2[0] + a2[1]) + (a2[2] + a2[3]);
    }
    __syncthreads();
    if (q == 0) {
        double s1 = 0.0, s2 = 0.0;
        for (int k = 0; k < 16; ++k) {
            s1 += sh[0][k][c];
            s2 += sh[1][k][c];
        }
        const double mu = s1 / N;
        double var = s2 / N - mu * mu;
        if (var < 0.0) var = 0.0;
        const float muf = (float)mu, isf = (float)(1.0 / sqrt(var + (double)eps));
        cf[0][c] = muf;
        cf[1][c] = isf;
        cf[2][c] = gamma[c];
        cf[3][c] = beta[c];
        if (blockIdx.x == 0) {
            mean_out[c] = muf;
            invstd_out[c] = isf;
            rmean[c] = (float)((1.0 - bn_mom) * rmean[c] + bn_mom * mu);
            rvar[c] = (float)((1.0 - bn_mom) * rvar[c] + bn_mom * var * N / (N - 1.0));
        }
    }
    __syncthreads();
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t * 4 < n; t += (long long)gridDim.x * blockDim.x) {
        const int c0 = (int)((t * 4) & 63);
        const float4 z = reinterpret_cast<const float4*>(Z)[t];
        float v[4] = {z.x, z.y, z.z, z.w};
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (skip) s = reinterpret_cast<const float4*>(skip)[t];
        const float sk[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float y = (v[k] - cf[0][c0 + k]) * cf[1][c0 + k] * cf[2][c0 + k] + cf[3][c0 + k];
            if (skip) y += sk[k];
            v[k] = y > 0.0f ? y : 0.0f;
        }
        reinterpret_cast<float4*>(A)[t] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// ---- BN backward finalisation: dgamma = sum m*xhat, dbeta = sum m; dx coefficients -----------------
// Channels c >= split: gamma2 / ggamma2 / gbeta2 [c - split] (both heads in one launch, as k_bn_fwd_fin).
__global__ __launch_bounds__(1024) void k_bn_bwd_fin(const float* part, int nwg, int pstride, int coff, int C, double N,
                             const float* gamma, const float* invstd, float* ggamma, float* gbeta,
                             float* c1, float* mm, float* mx, int split, const float* gamma2, float* ggamma2,
                             float* gbeta2) {
    __shared__ double sh[2][16][64];
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
        double a1[4] = {0.0, 0.0, 0.0, 0.0}, a2[4] = {0.0, 0.0, 0.0, 0.0};
        int w = q;
        for (; w + 48 < nwg; w += 64) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a1[u] += part[(size_t)(w + 16 * u) * 2 * pstride + coff + c];
                a2[u] += part[(size_t)(w + 16 * u) * 2 * pstride + pstride + coff + c];
            }
        }
        for (; w < nwg; w += 16) {
            a1[0] += part[(size_t)w * 2 * pstride + coff + c];
            a2[0] += part[(size_t)w * 2 * pstride + pstride + coff + c];
        }
        s1 = (a1[0] + a1[1]) + (a1[2] + a1[3]);
        s2 = (a2[0] + a2[1]) + (a2[2] + a2[3]);
    }
    sh[0][q][c] = s1;
    sh[1][q][c] = s2;
    __syncthreads();
    if (q == 0 && c < C) {
        s1 = 0.0;
        s2 = 0.0;
        for (int k = 0; k < 16; ++k) {
            s1 += sh[0][k][c];
            s2 += sh[1][k][c];
        }
        const bool lo = c < split;
        (lo ? gbeta + c : gbeta2 + (c - split))[0] = (float)s1;
        (lo ? ggamma + c : ggamma2 + (c - split))[0] = (float)s2;
        c1[c] = (lo ? gamma[c] : gamma2[c - split]) * invstd[c];
        mm[c] = (float)(s1 / N);
        mx[c] = (float)(s2 / N);
    }
}

// dZ = gamma*invstd * (m - mean(m) - xhat * mean(m*xhat)); per-(4U)-row partial sums of dZ (conv bias grad)
template <int U>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const float* M, const float* Z, const float* mean,
                                                      const float* invstd, const float* c1, const float* mm,
                                                      const float* mx, float* dZ, float* part, int R) {
    __shared__ float sh[4][64];
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int r0 = blockIdx.x * 4 * U;
    const float mu = mean[c], is = invstd[c], k1 = c1[c], k2 = mm[c], k3 = mx[c];
    float s = 0.0f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int r = r0 + q + 4 * u;
        if (r < R) {
            const size_t o = (size_t)r * kC + c;
            const float xh = (Z[o] - mu) * is;
            const float d = k1 * (M[o] - k2 - xh * k3);
            dZ[o] = d;
            s += d;
        }
    }
    sh[q][c] = s;
    __syncthreads();
    if (q == 0) part[(size_t)blockIdx.x * 64 + c] = sh[0][c] + sh[1][c] + sh[2][c] + sh[3][c];
}

// ---- weight gradient: per (tap, square, row split z) partial D[co][ci] = sum_b dZ[sq,b][co] * X[nbr,b][ci]
// v_mfma_f32_32x32x2_f32: lane l supplies A[m = l&31][k = l>>5] and B[k = l>>5][n = l&31], so one
// k-pair = two rows, read as 128-B row segments. A wave owns the whole 64 x (32*NNT) tile (2 x NNT
// accumulators); the 4 waves of a workgroup take interleaved row pairs and are summed in LDS.
#ifndef OAZ_WSPLIT
#define OAZ_WSPLIT 2
#endif
constexpr int kWSplit = OAZ_WSPLIT;  // row splits per (tap, square) (-DOAZ_WSPLIT: A/B variants)
template <int NNT>  // input-channel tiles of 32 (2 for 64 channels, 1 for the padded 32)
__global__ __launch_bounds__(256) void k_wgrad(const float* dZ, const float* X, int B, float* part) {
    __shared__ float red[3][64 * 64];
    const int sq = blockIdx.x, t = blockIdx.y, zs = blockIdx.z;
    const int nb = nbr(sq, t);
    if (nb < 0) return;
    constexpr int xrs = 32 * NNT;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    const int rows = B / kWSplit, r0 = zs * rows;
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    f32x16 acc[2][NNT];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < NNT; ++n) acc[m][n] = f32x16{};
    const float* pa = dZ + (size_t)(sq * B + r0 + h) * kC + c;
    const float* pb = X + (size_t)(nb * B + r0 + h) * xrs + c;
    float a[4][2], b[4][NNT], an[4][2], bn[4][NNT];
    auto load = [&](int k, float (&aa)[4][2], float (&bb)[4][NNT]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int kk = k + 8 * u;
            const bool ok = kk < rows;
#pragma unroll
            for (int m = 0; m < 2; ++m) aa[u][m] = ok ? pa[(size_t)kk * kC + 32 * m] : 0.0f;
#pragma unroll
            for (int n = 0; n < NNT; ++n) bb[u][n] = ok ? pb[(size_t)kk * xrs + 32 * n] : 0.0f;
        }
    };
    load(2 * wave, a, b);
    for (int k = 2 * wave; k < rows; k += 32) {  // 4 row pairs per iteration; next ones prefetched
        if (k + 32 < rows) load(k + 32, an, bn);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < NNT; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][m], b[u][n], acc[m][n], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int m = 0; m < 2; ++m) a[u][m] = an[u][m];
#pragma unroll
            for (int n = 0; n < NNT; ++n) b[u][n] = bn[u][n];
        }
    }
    // D layout: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
    if (wave > 0) {
        float* dst = red[wave - 1];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < NNT; ++n)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
                    dst[row * xrs + 32 * n + c] = acc[m][n][r];
                }
    }
    __syncthreads();
    if (wave == 0) {
        float* out = part + ((size_t)(t * 25 + sq) * kWSplit + zs) * kC * xrs;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < NNT; ++n)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int o = row * xrs + 32 * n + c;
                    out[o] = acc[m][n][r] + red[0][o] + red[1][o] + red[2][o];
                }
    }
}

// grad_w[co][ci][tap] (canonical [co][cin][3][3]) = sum over on-board squares and row splits.
// Threads run ci-fastest so the partial reads coalesce.
__global__ void k_wgrad_reduce(const float* part, int xrs, int cin, float* gw) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= 9 * kC * cin) return;
    const int ci = id % cin, co = (id / cin) % kC, t = id / (cin * kC);
    const float* p = part + ((size_t)t * 25 * kWSplit * kC + co) * xrs + ci;
    float s[kWSplit] = {};
#pragma unroll
    for (int sq = 0; sq < 25; ++sq) {  // predicated, fully unrolled: all loads in flight
        const bool ok = nbr(sq, t) >= 0;
#pragma unroll
        for (int zs = 0; zs < kWSplit; ++zs) s[zs] += ok ? p[(size_t)(sq * kWSplit + zs) * kC * xrs] : 0.0f;
    }
    float tot = 0.0f;
#pragma unroll
    for (int zs = 0; zs < kWSplit; ++zs) tot += s[zs];
    gw[((size_t)co * cin + ci) * 9 + t] = tot;
}

// ---- heads -------------------------------------------------------------------------------------
struct HeadOff {  // float offsets into the parameter / gradient blob
    int vcw, vcb, vg, vb, vrm, vrv, l1w, l1b, l2w, l2b;
    int pcw, pcb, pg, pb, prm, prv, plw, plb;
};

// zv = vh_conv(A) (1x1, 64 -> 1), zp = policy_conv(A) (64 -> 2); per-256-row BN partials
__global__ __launch_bounds__(256) void k_head_conv(const float* A, const float* P, HeadOff o, float* hz,
                                                   float* part, int R) {
    __shared__ float sh[4][6];
    const int r = blockIdx.x * 256 + threadIdx.x;
    float v[3] = {0.0f, 0.0f, 0.0f};
    if (r < R) {
        const float4* row = reinterpret_cast<const float4*>(A + (size_t)r * kC);
        float a0 = P[o.vcb], a1 = P[o.pcb], a2 = P[o.pcb + 1];
        for (int k = 0; k < 16; ++k) {
            const float4 x = row[k];
            const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 4 * k + j;
                a0 += P[o.vcw + c] * xs[j];
                a1 += P[o.pcw + c] * xs[j];
                a2 += P[o.pcw + 64 + c] * xs[j];
            }
        }
        v[0] = a0;
        v[1] = a1;
        v[2] = a2;
        *reinterpret_cast<float4*>(hz + (size_t)r * 4) = make_float4(a0, a1, a2, 0.0f);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float s1 = wave_sum(v[j]), s2 = wave_sum(v[j] * v[j]);
        if (lane == 0) {
            sh[wave][j] = s1;
            sh[wave][3 + j] = s2;
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int j = threadIdx.x;
        const float s = sh[0][j] + sh[1][j] + sh[2][j] + sh[3][j];
        part[(size_t)blockIdx.x * 8 + (j < 3 ? j : 4 + j - 3)] = s;  // [nwg][2][4]
    }
}

struct HeadStats {  // head BN batch statistics (channel 0 = value, 1..2 = policy)
    float mean[3], invstd[3];
    float c1[3], mm[3], mx[3];
};

// Value MLP (25 -> 64 -> 1, tanh), policy linear (50 -> 50) + softmax, alphaloss terms
// (net.rs:234-243) and their backward down to the head BN outputs. One wave (64 lanes) per sample,
// kHS = 4 samples per workgroup: at batch 512 that is 128 workgroups, and each lane's dependent
// chains of LDS reads are a quarter of a 16-lane-per-sample layout's (one wave per SIMD cannot hide
// them; the kernel is on the step's critical path).
// Q16: with value_loss_broadcast the value loss is mean_{i,j} (z_j - v_i)^2 over [B,B].
constexpr int kHS = 4;           // samples per workgroup
constexpr int kTPS = 256 / kHS;  // lanes per sample (a whole wave)
__device__ __forceinline__ float sumT(float v) {
#pragma unroll
    for (int o = 1; o < kTPS; o <<= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float maxT(float v) {
#pragma unroll
    for (int o = 1; o < kTPS; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

__global__ __launch_bounds__(256) void k_head_sample(const float* hz, const float* hst_mean, const float* hst_inv,
                                                     const float* P, HeadOff o, const float* pi, const float* z,
                                                     int B, int broadcast, float* g3, float* part_bn,
                                                     float* part_w, float* part_loss) {
    __shared__ float W[kHeadW];  // l1w[64][25] l1b[64] l2w[64] l2b | plw[50][50] plb[50]
    __shared__ float hv[kHS][25], h1[kHS][64], dh1[kHS][64], hp[kHS][50], dl[kHS][50], du[kHS];
    __shared__ float red[4][8];
    const int tid = threadIdx.x, j = tid % kTPS, sl = tid / kTPS, lane = tid & 63, wave = tid >> 6;
    for (int k = tid; k < kHeadVW; k += 256) W[k] = P[o.l1w + k];
    for (int k = tid; k < 2550; k += 256) W[kHeadVW + k] = P[o.plw + k];
    float sz = 0.0f, sz2 = 0.0f;
    if (broadcast) {  // batch sums of z (every workgroup; B floats)
        for (int k = tid; k < B; k += 256) {
            sz += z[k];
            sz2 += z[k] * z[k];
        }
        sz = wave_sum(sz);
        sz2 = wave_sum(sz2);
        if (lane == 0) {
            red[wave][0] = sz;
            red[wave][1] = sz2;
        }
    }
    __syncthreads();
    if (broadcast) {
        sz = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        sz2 = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    }
    const float* l1w = W;
    const float* l1b = W + 1600;
    const float* l2w = W + 1664;
    const float l2b = W[1728];
    const float* plw = W + kHeadVW;
    const float* plb = plw + 2500;
    const int b = blockIdx.x * kHS + sl;
    const bool ok = b < B;
    const float vm = hst_mean[0], vi = hst_inv[0], vg = P[o.vg], vb = P[o.vb];
    for (int sq = j; sq < 25; sq += kTPS) {
        float y = 0.0f;
        if (ok) y = (hz[(size_t)(sq * B + b) * 4] - vm) * vi * vg + vb;
        hv[sl][sq] = y > 0.0f ? y : 0.0f;
    }
    for (int k = j; k < 50; k += kTPS) {
        const int c = k / 25, sq = k % 25;
        float y = 0.0f;
        if (ok) y = (hz[(size_t)(sq * B + b) * 4 + 1 + c] - hst_mean[1 + c]) * hst_inv[1 + c] * P[o.pg + c] + P[o.pb + c];
        hp[sl][k] = y > 0.0f ? y : 0.0f;
    }
    __syncthreads();
    // value MLP forward
    float up = 0.0f;
    for (int oo = j; oo < 64; oo += kTPS) {
        float a = l1b[oo];
        for (int sq = 0; sq < 25; ++sq) a += l1w[oo * 25 + sq] * hv[sl][sq];
        a = a > 0.0f ? a : 0.0f;
        h1[sl][oo] = a;
        up += l2w[oo] * a;
    }
    const float v = tanhf(sumT(up) + l2b);
    // policy linear + softmax
    constexpr int NQ = (50 + kTPS - 1) / kTPS;  // policy entries per lane
    float lg[NQ];
    float mxl = -INFINITY;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int jj = j + kTPS * q;
        lg[q] = -INFINITY;
        if (jj < 50) {
            float a = plb[jj];
            for (int k = 0; k < 50; ++k) a += plw[jj * 50 + k] * hp[sl][k];
            lg[q] = a;
            mxl = fmaxf(mxl, a);
        }
    }
    mxl = maxT(mxl);
    float se = 0.0f, spi = 0.0f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int jj = j + kTPS * q;
        if (jj < 50) {
            lg[q] = expf(lg[q] - mxl);
            se += lg[q];
            spi += ok ? pi[(size_t)b * 50 + jj] : 0.0f;
        }
    }
    se = sumT(se);
    spi = sumT(spi);
    const float inv25B = 1.0f / (25.0f * (float)B);
    float lp = 0.0f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int jj = j + kTPS * q;
        if (jj < 50) {
            const float p = lg[q] / se;
            const float t = ok ? pi[(size_t)b * 50 + jj] : 0.0f;
            if (t != 0.0f) lp -= t * logf(p);
            dl[sl][jj] = ok ? (p * spi - t) * inv25B : 0.0f;
        }
    }
    lp = sumT(lp) * inv25B;
    // value loss and d/dv
    const float fB = (float)B;
    float lv = 0.0f, dv = 0.0f;
    if (ok) {
        if (broadcast) {
            lv = (sz2 - 2.0f * v * sz + fB * v * v) / (fB * fB);
            dv = 2.0f * (fB * v - sz) / (fB * fB);
        } else {
            const float d = v - z[b];
            lv = d * d / fB;
            dv = 2.0f * d / fB;
        }
    }
    const float duv = dv * (1.0f - v * v);
    if (j == 0) du[sl] = duv;
    for (int oo = j; oo < 64; oo += kTPS) dh1[sl][oo] = h1[sl][oo] > 0.0f ? duv * l2w[oo] : 0.0f;
    __syncthreads();
    // backward into the head BN outputs
    float bnp[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // (sum g, sum g*xhat) x channel
    if (ok) {
        for (int sq = j; sq < 25; sq += kTPS) {
            float d = 0.0f;
            for (int oo = 0; oo < 64; ++oo) d += l1w[oo * 25 + sq] * dh1[sl][oo];
            const float g = hv[sl][sq] > 0.0f ? d : 0.0f;
            const size_t r = (size_t)(sq * B + b);
            g3[r * 4] = g;
            bnp[0] += g;
            bnp[1] += g * ((hz[r * 4] - vm) * vi);
        }
        for (int k = j; k < 50; k += kTPS) {
            float d = 0.0f;
            for (int jj = 0; jj < 50; ++jj) d += plw[jj * 50 + k] * dl[sl][jj];
            const float g = hp[sl][k] > 0.0f ? d : 0.0f;
            const int c = k / 25, sq = k % 25;
            const size_t r = (size_t)(sq * B + b);
            g3[r * 4 + 1 + c] = g;
            bnp[2 + 2 * c] += g;
            bnp[3 + 2 * c] += g * ((hz[r * 4 + 1 + c] - hst_mean[1 + c]) * hst_inv[1 + c]);
        }
    }
    // workgroup partials: BN sums and losses (lv, lp are per sample: count them on lane j == 0)
    float vals[8] = {bnp[0], bnp[2], bnp[4], bnp[1], bnp[3], bnp[5], j == 0 ? lv : 0.0f, j == 0 ? lp : 0.0f};
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float s = wave_sum(vals[k]);
        if (lane == 0) red[wave][k] = s;
    }
    __syncthreads();
    if (tid < 8) {
        const float s = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
        if (tid < 3) part_bn[(size_t)blockIdx.x * 8 + tid] = s;            // sum g
        else if (tid < 6) part_bn[(size_t)blockIdx.x * 8 + 4 + tid - 3] = s;  // sum g*xhat
        else part_loss[blockIdx.x * 2 + tid - 6] = s;
    }
    // weight-gradient partials over this workgroup's samples
    float* pw = part_w + (size_t)blockIdx.x * kHeadW;
    for (int e = tid; e < kHeadW; e += 256) {
        float s = 0.0f;
        if (e < 1600) {  // vh_linear1.weight [64][25]
            const int oo = e / 25, sq = e % 25;
            for (int k = 0; k < kHS; ++k) s += dh1[k][oo] * hv[k][sq];
        } else if (e < 1664) {  // vh_linear1.bias
            for (int k = 0; k < kHS; ++k) s += dh1[k][e - 1600];
        } else if (e < 1728) {  // vh_linear2.weight [1][64]
            for (int k = 0; k < kHS; ++k) s += du[k] * h1[k][e - 1664];
        } else if (e == 1728) {  // vh_linear2.bias
            for (int k = 0; k < kHS; ++k) s += du[k];
        } else if (e < kHeadVW + 2500) {  // ph_linear2.weight [50][50]
            const int jj = (e - kHeadVW) / 50, kk = (e - kHeadVW) % 50;
            for (int k = 0; k < kHS; ++k) s += dl[k][jj] * hp[k][kk];
        } else {  // ph_linear2.bias
            for (int k = 0; k < kHS; ++k) s += dl[k][e - kHeadVW - 2500];
        }
        pw[e] = s;
    }
}

// out[j] = sum_w part[w*pstride + src + j], j < width (64 columns x 16 row groups per workgroup)
__global__ __launch_bounds__(1024) void k_colsum(const float* part, int nwg, int pstride, int src, int width,
                                                 float* out) {
    __shared__ float sh[16][64];
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c;
    float s = 0.0f;
    if (j < width)
        for (int w = q; w < nwg; w += 16) s += part[(size_t)w * pstride + src + j];
    sh[q][c] = s;
    __syncthreads();
    if (q == 0 && j < width) {
        float t = 0.0f;
        for (int k = 0; k < 16; ++k) t += sh[k][c];
        out[j] = t;
    }
}

// Loss accumulators (double) += this step's sums (one wave: lane-strided partials, then a fixed-order
// tree over the lanes)
__global__ void k_loss_acc(const float* part_loss, int nwg, double* acc) {
    const int lane = threadIdx.x;
    double v = 0.0, p = 0.0;
    for (int w = lane; w < nwg; w += 64) {
        v += part_loss[2 * w];
        p += part_loss[2 * w + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        v += __shfl_xor(v, o);
        p += __shfl_xor(p, o);
    }
    if (lane == 0) {
        acc[0] += v;
        acc[1] += p;
        acc[2] += 1.0;
    }
}

// Per trunk row: head BN backward -> dA = wv * dzv + wp0 * dzp0 + wp1 * dzp1; m = dA * (A > 0);
// partials: sum m, sum m*xhat (last trunk BN), head conv weight/bias grads.
__global__ __launch_bounds__(256) void k_head_bwd_rows(const float* A, const float* Z, const float* mean,
                                                       const float* invstd, const float* hz, const float* g3,
                                                       const float* hst_mean, const float* hst_inv,
                                                       const float* hc1, const float* hmm, const float* hmx,
                                                       const float* P, HeadOff o, float* M, float* part_bn,
                                                       float* part_hc, int R) {
    __shared__ float sh[4][8][64];
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int r0 = blockIdx.x * 64;
    const float wv = P[o.vcw + c], wp0 = P[o.pcw + c], wp1 = P[o.pcw + 64 + c];
    const float mu = mean[c], is = invstd[c];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // sum m, sum m*xh, dwv, dwp0, dwp1, dbv, dbp0, dbp1
    for (int r = r0 + q; r < min(r0 + 64, R); r += 4) {
        float dz[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float xh = (hz[(size_t)r * 4 + k] - hst_mean[k]) * hst_inv[k];
            dz[k] = hc1[k] * (g3[(size_t)r * 4 + k] - hmm[k] - xh * hmx[k]);
        }
        const size_t off = (size_t)r * kC + c;
        const float a = A[off];
        const float dA = wv * dz[0] + wp0 * dz[1] + wp1 * dz[2];
        const float m = a > 0.0f ? dA : 0.0f;
        M[off] = m;
        acc[0] += m;
        acc[1] += m * ((Z[off] - mu) * is);
        acc[2] += dz[0] * a;
        acc[3] += dz[1] * a;
        acc[4] += dz[2] * a;
        acc[5] += dz[0];
        acc[6] += dz[1];
        acc[7] += dz[2];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[q][k][c] = acc[k];
    __syncthreads();
    if (q == 0) {
        float s[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = sh[0][k][c] + sh[1][k][c] + sh[2][k][c] + sh[3][k][c];
        part_bn[(size_t)blockIdx.x * 128 + c] = s[0];
        part_bn[(size_t)blockIdx.x * 128 + 64 + c] = s[1];
        float* ph = part_hc + (size_t)blockIdx.x * kHConvW;  // vh_conv w[64] b | policy_conv w[2][64] b[2]
        ph[c] = s[2];
        ph[65 + c] = s[3];
        ph[65 + 64 + c] = s[4];
        if (c == 0) {
            ph[64] = s[5];
            ph[65 + 128] = s[6];
            ph[65 + 129] = s[7];
        }
    }
}

// ---- optimiser + weight packing -------------------------------------------------------------------
struct ConvTab {  // conv weight ranges of the blob and their packed copies (written by k_sgd)
    int n;
    int off[kMaxConv], cin[kMaxConv];
    float* wf[kMaxConv];
    float* wd[kMaxConv];
};

// SGD (torch semantics, dampening 0): d = g*scale + wd*p; buf = mom*buf + d; p -= lr*buf.
// Conv weights are also scattered straight into the packed fwd / dgrad layouts of k_pack.
__global__ void k_sgd(float* p, const float* g, float* buf, const uint8_t* mask, long long n, float lr,
                      float mom, float wd, float scale, ConvTab tab) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !mask[i]) return;
    const float d = g[i] * scale + wd * p[i];
    const float bb = mom * buf[i] + d;
    buf[i] = bb;
    const float np = p[i] - lr * bb;
    p[i] = np;
    for (int l = 0; l < tab.n; ++l) {
        const int cin = tab.cin[l];
        const long long rel = i - tab.off[l];
        if (rel < 0 || rel >= (long long)kC * cin * 9) continue;
        const int t = (int)(rel % 9), ci = (int)((rel / 9) % cin), co = (int)(rel / (9 * cin));
        const int chunks = cin == kC ? 4 : 2;
        {
            const int gg = ci >> 4, kq = (ci & 15) >> 2, j = ci & 3, nt = co >> 4, lane = (co & 15) + 16 * kq;
            tab.wf[l][((((size_t)t * chunks + gg) * 4 + nt) * 64 + lane) * 4 + j] = np;
        }
        if (tab.wd[l]) {
            const int gg = co >> 4, kq = (co & 15) >> 2, j = co & 3, nt = ci >> 4, lane = (ci & 15) + 16 * kq;
            tab.wd[l][((((size_t)(8 - t) * 4 + gg) * 4 + nt) * 64 + lane) * 4 + j] = np;
        }
        break;
    }
}

// Packed conv weights: float4 index ((t*chunks + g)*4 + nt)*64 + lane holds, for output channel
// nt*16 + (lane&15), input channels 16g + 4*(lane>>4) + {0..3}.
//   fwd:   W[co][ci][t]            (co = output, ci = input; ci >= cin -> 0)
//   dgrad: W[ci'][co'][8 - t]      (output = original input channel, input = original output)
__global__ void k_pack(const float* W, int cin, int chunks, float4* wf, float4* wd) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= 9 * chunks * 256) return;
    const int lane = id & 63, nt = (id >> 6) & 3, g = (id >> 8) % chunks, t = (id >> 8) / chunks;
    const int oc = nt * 16 + (lane & 15), ic0 = 16 * g + 4 * (lane >> 4);
    float v[4], d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ic = ic0 + j;
        v[j] = ic < cin ? W[((size_t)oc * cin + ic) * 9 + t] : 0.0f;
        d[j] = (wd && oc < cin) ? W[((size_t)ic * cin + oc) * 9 + (8 - t)] : 0.0f;
    }
    wf[id] = make_float4(v[0], v[1], v[2], v[3]);
    if (wd) wd[id] = make_float4(d[0], d[1], d[2], d[3]);
}

}  // namespace tr

using namespace tr;

// ---- host trainer ---------------------------------------------------------------------------------
struct Layout {
    size_t cw[kMaxConv], cb[kMaxConv], bg[kMaxConv], bb[kMaxConv], brm[kMaxConv], brv[kMaxConv];
    HeadOff h;
    size_t total;
};

static Layout make_layout(int blocks) {  // weights.py canonical_layout / VarStore order
    Layout L{};
    size_t p = 0;
    const int nconv = 1 + 2 * blocks;
    for (int l = 0; l < nconv; ++l) {
        const size_t cin = l == 0 ? kIn : kC;
        L.cw[l] = p; p += kC * cin * 9;
        L.cb[l] = p; p += kC;
        L.bg[l] = p; p += kC;
        L.bb[l] = p; p += kC;
        L.brm[l] = p; p += kC;
        L.brv[l] = p; p += kC;
    }
    HeadOff& h = L.h;
    h.vcw = (int)p; p += 64;
    h.vcb = (int)p; p += 1;
    h.vg = (int)p; p += 1;
    h.vb = (int)p; p += 1;
    h.vrm = (int)p; p += 1;
    h.vrv = (int)p; p += 1;
    h.l1w = (int)p; p += 64 * 25;
    h.l1b = (int)p; p += 64;
    h.l2w = (int)p; p += 64;
    h.l2b = (int)p; p += 1;
    h.pcw = (int)p; p += 128;
    h.pcb = (int)p; p += 2;
    h.pg = (int)p; p += 2;
    h.pb = (int)p; p += 2;
    h.prm = (int)p; p += 2;
    h.prv = (int)p; p += 2;
    h.plw = (int)p; p += 2500;
    h.plb = (int)p; p += 50;
    L.total = p;
    return L;
}

struct oaz_trainer {
    oaz_train_config cfg{};
    int device = 0;
    hipStream_t own = nullptr, st = nullptr;
    hipStream_t st2 = nullptr;  // weight-gradient stream: wgrad(l) overlaps dgrad(l) on st
    hipEvent_t ev_dz[2] = {}, ev_w[2] = {}, ev_h[2] = {}, ev_done = nullptr;
    Layout L{};
    int nconv = 0, maxB = 0;
    int cfin = -1;     // forward BN finalisation in k_bn_act_cfin (-1: one float4 per thread; A/B build: 0 = the
                       // separate k_bn_fwd_fin + k_bn_act launches, n > 0 = n workgroups)
    int conv_rg = 2;  // 16-row groups per conv workgroup (OAZ_CONV_RG=1|2|4 overrides; tuning knob)
    size_t nparam = 0;
    std::vector<void*> allocs;
    float *P = nullptr, *G = nullptr, *MOM = nullptr;
    uint8_t* mask = nullptr;
    float4 *wf[kMaxConv] = {}, *wd[kMaxConv] = {};
    float *X0 = nullptr, *Z[kMaxConv] = {}, *A[kMaxConv] = {}, *M[kMaxConv] = {}, *DZ[2] = {};
    float *mean[kMaxConv] = {}, *invstd[kMaxConv] = {}, *bcoef = nullptr;  // bcoef: c1, mm, mx [3][64]
    float *part = nullptr, *bpart[2] = {}, *wpart = nullptr;
    float *hz = nullptr, *g3 = nullptr, *hstat = nullptr;  // hstat: mean[3] invstd[3] c1[3] mm[3] mx[3]
    float *hpart = nullptr, *hwpart = nullptr, *hlpart = nullptr, *hcpart = nullptr;
    float *pi = nullptr, *z = nullptr;
    const oaz_sample* samples = nullptr;
    oaz_sample* owned_samples = nullptr;
    size_t n_samples = 0, owned_cap = 0;
    int32_t* idx = nullptr;
    int n_batches = 0, batch = 0;
    size_t idx_cap = 0;
    double* loss_acc = nullptr;
    int32_t* cur = nullptr;  // current batch number (device)
    // one captured SGD step (gather -> ... -> SGD -> batch+1), replayed by oaz_trainer_train
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    const void* graph_key[3] = {nullptr, nullptr, nullptr};
    int graph_batch = 0;

    template <class T>
    int alloc(T*& p, size_t count) {
        void* q = nullptr;
        HIP_TRY(hipMalloc(&q, count * sizeof(T) + 16));
        HIP_TRY(hipMemsetAsync(q, 0, count * sizeof(T) + 16, own));  // ordered before the trainer's work (create syncs)
        allocs.push_back(q);
        p = (T*)q;
        return 0;
    }
    ~oaz_trainer() {
        if (owned_samples) (void)hipFree(owned_samples);
        if (idx) (void)hipFree(idx);
        for (void* q : allocs) (void)hipFree(q);
        for (int k = 0; k < 2; ++k) {
            if (ev_dz[k]) (void)hipEventDestroy(ev_dz[k]);
            if (ev_w[k]) (void)hipEventDestroy(ev_w[k]);
        }
        if (ev_done) (void)hipEventDestroy(ev_done);
        for (hipEvent_t ev : ev_h)
            if (ev) (void)hipEventDestroy(ev);
        if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
        if (graph) (void)hipGraphDestroy(graph);
        if (st2) (void)hipStreamDestroy(st2);
        if (own) (void)hipStreamDestroy(own);
    }
};

extern "C" void oaz_train_config_default(oaz_train_config* c) {
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->blocks = 5;
    c->max_batch = 512;
    c->learning_rate = 5e-3;
    c->momentum = 0.9;
    c->weight_decay = 1e-4;
    c->bn_momentum = 0.1;
    c->bn_eps = 1e-5;
    c->value_loss_broadcast = 1;
}

extern "C" oaz_trainer* oaz_trainer_create(const oaz_train_config* cfg, int device) {
    if (!cfg || cfg->blocks < 0 || cfg->blocks > 16 || cfg->max_batch < 16 || cfg->max_batch % 16 ||
        cfg->max_batch > (1 << 16)) {
        oaz_set_err(OAZ_ERR_ARG, "trainer: blocks in [0,16], max_batch a multiple of 16 in [16, 65536]");
        return nullptr;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        oaz_set_err(OAZ_ERR_NO_DEVICE, "trainer: no HIP device %d", device);
        return nullptr;
    }
    DeviceScope dev_scope_(device);  // the caller's current device is restored on return
    if (dev_scope_.rc != hipSuccess) {
        oaz_set_err(OAZ_ERR_NO_DEVICE, "trainer: hipSetDevice(%d) failed", device);
        return nullptr;
    }
    oaz_trainer* t = new oaz_trainer();
    t->cfg = *cfg;
    t->device = device;
    t->nconv = 1 + 2 * cfg->blocks;
    t->maxB = cfg->max_batch;
    t->L = make_layout(cfg->blocks);
#if OAZ_AB  // A/B build only: conv row-group override
    if (const char* e = getenv("OAZ_CONV_RG")) {
        const int v = atoi(e);
        if (v == 1 || v == 2 || v == 4) t->conv_rg = v;
    }
    if (const char* e = getenv("OAZ_TRAIN_CFIN")) t->cfin = atoi(e) > 0 ? atoi(e) : 0;
#endif
    t->nparam = t->L.total;
    const size_t R = (size_t)t->maxB * 25;
    auto fail = [&]() -> oaz_trainer* { delete t; return nullptr; };
    bool ev_ok = hipStreamCreateWithFlags(&t->st2, hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&t->ev_done, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; k < 2 && ev_ok; ++k)
        ev_ok = hipEventCreateWithFlags(&t->ev_dz[k], hipEventDisableTiming) == hipSuccess &&
                hipEventCreateWithFlags(&t->ev_w[k], hipEventDisableTiming) == hipSuccess &&
                hipEventCreateWithFlags(&t->ev_h[k], hipEventDisableTiming) == hipSuccess;
    if (!ev_ok || hipStreamCreateWithFlags(&t->own, hipStreamNonBlocking) != hipSuccess) {
        oaz_set_err(OAZ_ERR_HIP, "trainer: stream");
        return fail();
    }
    t->st = t->own;
    if (t->alloc(t->P, t->nparam) || t->alloc(t->G, t->nparam) || t->alloc(t->MOM, t->nparam) ||
        t->alloc(t->mask, t->nparam))
        return fail();
    for (int l = 0; l < t->nconv; ++l) {
        const int chunks = l == 0 ? 2 : 4;
        if (t->alloc(t->wf[l], (size_t)9 * chunks * 256)) return fail();
        if (l > 0 && t->alloc(t->wd[l], (size_t)9 * chunks * 256)) return fail();
        if (t->alloc(t->Z[l], R * kC) || t->alloc(t->A[l], R * kC) || t->alloc(t->M[l], R * kC) ||
            t->alloc(t->mean[l], 64) || t->alloc(t->invstd[l], 64))
            return fail();
    }
    const size_t nwg_conv = R / 16;
    if (t->alloc(t->X0, R * kInPad) || t->alloc(t->DZ[0], R * kC) || t->alloc(t->DZ[1], R * kC) || t->alloc(t->bcoef, 3 * 64) ||
        t->alloc(t->part, nwg_conv * 128) || t->alloc(t->bpart[0], (R + 15) / 16 * 64) || t->alloc(t->bpart[1], (R + 15) / 16 * 64) ||
        t->alloc(t->wpart, (size_t)9 * 25 * kWSplit * 64 * 64) || t->alloc(t->hz, R * 4) || t->alloc(t->g3, R * 4) ||
        t->alloc(t->hstat, 16) || t->alloc(t->hpart, ((R + 255) / 256 + (size_t)t->maxB / kHS + 1) * 8) ||
        t->alloc(t->hwpart, ((size_t)t->maxB / kHS + 1) * kHeadW) ||
        t->alloc(t->hlpart, ((size_t)t->maxB / kHS + 1) * 2) ||
        t->alloc(t->hcpart, ((R + 63) / 64) * (size_t)kHConvW) || t->alloc(t->pi, (size_t)t->maxB * 50) ||
        t->alloc(t->z, (size_t)t->maxB) || t->alloc(t->loss_acc, 4) || t->alloc(t->cur, 1))
        return fail();
    std::vector<uint8_t> mask(t->nparam, 1);
    for (int l = 0; l < t->nconv; ++l)
        for (int c = 0; c < 64; ++c) mask[t->L.brm[l] + c] = mask[t->L.brv[l] + c] = 0;
    mask[t->L.h.vrm] = mask[t->L.h.vrv] = 0;
    mask[t->L.h.prm] = mask[t->L.h.prm + 1] = mask[t->L.h.prv] = mask[t->L.h.prv + 1] = 0;
    if (hipMemcpyAsync(t->mask, mask.data(), t->nparam, hipMemcpyHostToDevice, t->own) != hipSuccess ||
        hipStreamSynchronize(t->own) != hipSuccess) {  // the zero fills and the mask landed before any step
        oaz_set_err(OAZ_ERR_HIP, "trainer: mask upload");
        return fail();
    }
    return t;
}

extern "C" void oaz_trainer_destroy(oaz_trainer* t) {
    if (!t) return;
    DeviceScope dev_scope_(t->device);
    (void)hipDeviceSynchronize();
    delete t;
}

extern "C" int oaz_trainer_set_stream(oaz_trainer* t, void* stream) {
    if (!t) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    t->st = stream ? (hipStream_t)stream : t->own;
    return 0;
}

static int repack(oaz_trainer* t) {
    for (int l = 0; l < t->nconv; ++l) {
        const int chunks = l == 0 ? 2 : 4, cin = l == 0 ? kIn : kC;
        const int n = 9 * chunks * 256;
        hipLaunchKernelGGL(k_pack, dim3((n + 255) / 256), dim3(256), 0, t->st, t->P + t->L.cw[l], cin, chunks,
                           t->wf[l], t->wd[l]);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int oaz_trainer_set_weights(oaz_trainer* t, const float* blob, size_t n) {
    if (!t || !blob || n != t->nparam) return oaz_set_err(OAZ_ERR_ARG, "trainer: need %zu floats", t ? t->nparam : 0);
    OAZ_ON_DEVICE(t->device);
    HIP_TRY(hipMemcpyAsync(t->P, blob, n * sizeof(float), hipMemcpyHostToDevice, t->st));
    HIP_TRY(hipMemsetAsync(t->MOM, 0, n * sizeof(float), t->st));
    if (int rc = repack(t)) return rc;
    HIP_TRY(hipStreamSynchronize(t->st));
    return 0;
}

extern "C" int oaz_trainer_get_weights(oaz_trainer* t, float* blob, size_t n) {
    if (!t || !blob || n != t->nparam) return oaz_set_err(OAZ_ERR_ARG, "trainer: need %zu floats", t ? t->nparam : 0);
    OAZ_ON_DEVICE(t->device);
    HIP_TRY(hipMemcpyAsync(blob, t->P, n * sizeof(float), hipMemcpyDeviceToHost, t->st));
    HIP_TRY(hipStreamSynchronize(t->st));
    return 0;
}

extern "C" int oaz_trainer_save_ot(oaz_trainer* t, const char* path) {
    if (!t || !path) return oaz_set_err(OAZ_ERR_ARG, "trainer_save_ot: null");
    std::vector<float> blob(t->nparam);
    if (int rc = oaz_trainer_get_weights(t, blob.data(), blob.size())) return rc;
    return oaz_ot_write(path, blob.data(), blob.size(), t->cfg.blocks);
}

extern "C" int oaz_trainer_load_samples(oaz_trainer* t, const oaz_sample* s, size_t n) {
    if (!t || (!s && n)) return oaz_set_err(OAZ_ERR_ARG, "trainer: null samples");
    OAZ_ON_DEVICE(t->device);
    if (n > t->owned_cap) {
        HIP_TRY(hipStreamSynchronize(t->st));
        if (t->owned_samples) HIP_TRY(hipFree(t->owned_samples));
        t->owned_samples = nullptr;
        t->owned_cap = 0;
        HIP_TRY(hipMalloc(&t->owned_samples, n * sizeof(oaz_sample)));
        t->owned_cap = n;
    }
    if (n) HIP_TRY(hipMemcpyAsync(t->owned_samples, s, n * sizeof(oaz_sample), hipMemcpyHostToDevice, t->st));
    HIP_TRY(hipStreamSynchronize(t->st));
    t->samples = t->owned_samples;
    t->n_samples = n;
    return 0;
}

extern "C" int oaz_trainer_bind_device_samples(oaz_trainer* t, const oaz_sample* s, size_t n) {
    if (!t || (!s && n)) return oaz_set_err(OAZ_ERR_ARG, "trainer: null samples");
    t->samples = s;
    t->n_samples = n;
    return 0;
}

extern "C" int oaz_trainer_set_batches(oaz_trainer* t, const int32_t* idx, int n_batches, int batch) {
    if (!t || !idx || n_batches < 0 || batch < 16 || batch % 16 || batch > t->maxB)
        return oaz_set_err(OAZ_ERR_ARG, "trainer: batch must be a multiple of 16 in [16, %d]", t ? t->maxB : 0);
    const size_t n = (size_t)n_batches * batch;
    for (size_t i = 0; i < n; ++i)
        if (idx[i] < 0 || (size_t)idx[i] >= t->n_samples)
            return oaz_set_err(OAZ_ERR_ARG, "trainer: index %d out of range (%zu samples)", idx[i], t->n_samples);
    OAZ_ON_DEVICE(t->device);
    if (n > t->idx_cap) {
        HIP_TRY(hipStreamSynchronize(t->st));
        if (t->idx) HIP_TRY(hipFree(t->idx));
        t->idx = nullptr;
        t->idx_cap = 0;
        HIP_TRY(hipMalloc(&t->idx, n * sizeof(int32_t)));
        t->idx_cap = n;
    }
    if (n) HIP_TRY(hipMemcpyAsync(t->idx, idx, n * sizeof(int32_t), hipMemcpyHostToDevice, t->st));
    HIP_TRY(hipStreamSynchronize(t->st));
    t->n_batches = n_batches;
    t->batch = batch;
    return 0;
}

template <int MODE>
static void launch_conv(int ch, int rg, dim3 grid, hipStream_t st, const ConvArgs& a) {
#define OAZ_CONV(CHV, RGV) hipLaunchKernelGGL((k_conv<MODE, CHV, RGV>), grid, dim3(256), 0, st, a)
    if (ch == 2) {
        if (rg == 1) OAZ_CONV(2, 1); else if (rg == 2) OAZ_CONV(2, 2); else OAZ_CONV(2, 4);
    } else {
        if (rg == 1) OAZ_CONV(4, 1); else if (rg == 2) OAZ_CONV(4, 2); else OAZ_CONV(4, 4);
    }
#undef OAZ_CONV
}

static int backward(oaz_trainer* t, int bi) {
    const int B = t->batch, R = B * 25, NB = t->cfg.blocks, nl = t->nconv;
    const Layout& L = t->L;
    const HeadOff& h = L.h;
    hipStream_t st = t->st;
    float* P = t->P;
    float* G = t->G;
    const float bn_mom = (float)t->cfg.bn_momentum, eps = (float)t->cfg.bn_eps;
    const int rg = t->conv_rg, rows_wg = 16 * rg;
    const int nwg_conv = 25 * ((B + rows_wg - 1) / rows_wg);
    const dim3 conv_grid((B + rows_wg - 1) / rows_wg, 25);
    hipLaunchKernelGGL(k_gather, dim3((R + 51 * B + 255) / 256), dim3(256), 0, st, t->samples, t->idx, t->cur, bi, B,
                       t->X0, t->pi, t->z);
    // ---- forward
    for (int l = 0; l < nl; ++l) {
        ConvArgs a{};
        a.in = l == 0 ? t->X0 : t->A[l - 1];
        a.w = t->wf[l];
        a.bias = P + L.cb[l];
        a.out = t->Z[l];
        a.part = t->part;
        a.chunks = l == 0 ? 2 : 4;
        a.B = B;
        launch_conv<CONV_FWD>(l == 0 ? 2 : 4, rg, conv_grid, st, a);
        const float* skip = (l >= 2 && l % 2 == 0) ? t->A[l - 2] : nullptr;  // block output adds the block input
        const long long n = (long long)R * kC;
        if (t->cfin) {
            const unsigned nwg_act = t->cfin > 0 ? (unsigned)t->cfin : (unsigned)((n / 4 + 1023) / 1024);
            hipLaunchKernelGGL(k_bn_act_cfin, dim3(nwg_act), dim3(1024), 0, st, t->part, nwg_conv, (double)R,
                               P + L.brm[l], P + L.brv[l], bn_mom, eps, t->mean[l], t->invstd[l], t->Z[l],
                               P + L.bg[l], P + L.bb[l], skip, t->A[l], n);
            continue;
        }
        hipLaunchKernelGGL(k_bn_fwd_fin, dim3(1), dim3(1024), 0, st, t->part, nwg_conv, 64, 0, 64, (double)R,
                           P + L.brm[l], P + L.brv[l], bn_mom, eps, t->mean[l], t->invstd[l], 64, nullptr, nullptr);
        hipLaunchKernelGGL(k_bn_act, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, t->Z[l], t->mean[l],
                           t->invstd[l], P + L.bg[l], P + L.bb[l], skip, t->A[l], n);
    }
    (void)NB;
    // ---- heads
    const float* AL = t->A[nl - 1];
    const int nwg_hc = (R + 255) / 256;
    hipLaunchKernelGGL(k_head_conv, dim3(nwg_hc), dim3(256), 0, st, AL, P, h, t->hz, t->hpart, R);
    float* hmean = t->hstat;
    float* hinv = t->hstat + 3;
    float* hc1 = t->hstat + 6;
    float* hmm = t->hstat + 9;
    float* hmx = t->hstat + 12;
    hipLaunchKernelGGL(k_bn_fwd_fin, dim3(1), dim3(1024), 0, st, t->hpart, nwg_hc, 4, 0, 3, (double)R,
                       P + h.vrm, P + h.vrv, bn_mom, eps, hmean, hinv, 1, P + h.prm, P + h.prv);
    const int nwg_hs = (B + kHS - 1) / kHS;
    float* hbpart = t->hpart + (size_t)nwg_hc * 8;
    hipLaunchKernelGGL(k_head_sample, dim3(nwg_hs), dim3(256), 0, st, t->hz, hmean, hinv, P, h, t->pi, t->z, B,
                       t->cfg.value_loss_broadcast, t->g3, hbpart, t->hwpart, t->hlpart);
    // the losses and the heads' weight gradients are off the critical path: the weight-gradient stream
    // sums them (st waits for st2 before SGD, and the next step's head_sample, ev_done)
    HIP_TRY(hipEventRecord(t->ev_h[0], st));
    HIP_TRY(hipStreamWaitEvent(t->st2, t->ev_h[0], 0));
    hipLaunchKernelGGL(k_loss_acc, dim3(1), dim3(64), 0, t->st2, t->hlpart, nwg_hs, t->loss_acc);
    hipLaunchKernelGGL(k_colsum, dim3((kHeadVW + 63) / 64), dim3(1024), 0, t->st2, t->hwpart, nwg_hs, kHeadW, 0,
                       kHeadVW, G + h.l1w);
    hipLaunchKernelGGL(k_colsum, dim3((2550 + 63) / 64), dim3(1024), 0, t->st2, t->hwpart, nwg_hs, kHeadW, kHeadVW,
                       2550, G + h.plw);
    hipLaunchKernelGGL(k_bn_bwd_fin, dim3(1), dim3(1024), 0, st, hbpart, nwg_hs, 4, 0, 3, (double)R, P + h.vg,
                       hinv, G + h.vg, G + h.vb, hc1, hmm, hmx, 1, P + h.pg, G + h.pg, G + h.pb);
    const int nwg_rows = (R + 63) / 64;
    hipLaunchKernelGGL(k_head_bwd_rows, dim3(nwg_rows), dim3(256), 0, st, AL, t->Z[nl - 1], t->mean[nl - 1],
                       t->invstd[nl - 1], t->hz, t->g3, hmean, hinv, hc1, hmm, hmx, P, h, t->M[nl - 1], t->part,
                       t->hcpart, R);
    HIP_TRY(hipEventRecord(t->ev_h[1], st));
    HIP_TRY(hipStreamWaitEvent(t->st2, t->ev_h[1], 0));
    hipLaunchKernelGGL(k_colsum, dim3(2), dim3(1024), 0, t->st2, t->hcpart, nwg_rows, kHConvW, 0, 65, G + h.vcw);
    hipLaunchKernelGGL(k_colsum, dim3(3), dim3(1024), 0, t->st2, t->hcpart, nwg_rows, kHConvW, 65, 130, G + h.pcw);
    // ---- trunk backward; t->part holds the BN-backward partials of layer l (nwg, [2][64]).
    // dZ of layer l feeds both dgrad(l) (on st, the critical path) and wgrad(l) (on st2); dZ and
    // the bias partials are double-buffered so st never overwrites what st2 still reads.
    int nwg_part = nwg_rows;
    constexpr int kBwdU = 16;  // k_bn_bwd_apply rows per workgroup / 4 (4, 8, 32 measured slower)
    const int nwg_bwd = (R + 4 * kBwdU - 1) / (4 * kBwdU);
    bool used[2] = {false, false};
    for (int l = nl - 1; l >= 0; --l) {
        const int k = l & 1;
        float* c1 = t->bcoef;
        float* mm = t->bcoef + 64;
        float* mx = t->bcoef + 128;
        float* dz = t->DZ[k];
        if (used[k]) HIP_TRY(hipStreamWaitEvent(st, t->ev_w[k], 0));
        hipLaunchKernelGGL(k_bn_bwd_fin, dim3(1), dim3(1024), 0, st, t->part, nwg_part, 64, 0, 64, (double)R,
                           P + L.bg[l], t->invstd[l], G + L.bg[l], G + L.bb[l], c1, mm, mx, 64, nullptr,
                           nullptr, nullptr);
        hipLaunchKernelGGL(k_bn_bwd_apply<kBwdU>, dim3(nwg_bwd), dim3(256), 0, st, t->M[l], t->Z[l], t->mean[l],
                           t->invstd[l], c1, mm, mx, dz, t->bpart[k], R);
        // the weight gradient of layer l (second stream): it needs dz(l) and the layer's input X only, and runs
        // beside dgrad(l) (started after dgrad(l) instead, beside the next layer's BN kernels: 0.846 vs 0.764 ms
        // per step)
        auto wgrad = [&]() -> int {
            HIP_TRY(hipEventRecord(t->ev_dz[k], st));
            HIP_TRY(hipStreamWaitEvent(t->st2, t->ev_dz[k], 0));
            const float* X = l == 0 ? t->X0 : t->A[l - 1];
            if (l == 0)
                hipLaunchKernelGGL(k_wgrad<1>, dim3(25, 9, kWSplit), dim3(256), 0, t->st2, dz, X, B, t->wpart);
            else
                hipLaunchKernelGGL(k_wgrad<2>, dim3(25, 9, kWSplit), dim3(256), 0, t->st2, dz, X, B, t->wpart);
            const int cin = l == 0 ? kIn : kC;
            const int nred = 9 * kC * cin;
            hipLaunchKernelGGL(k_wgrad_reduce, dim3((nred + 255) / 256), dim3(256), 0, t->st2, t->wpart,
                               l == 0 ? kInPad : kC, cin, G + L.cw[l]);
            hipLaunchKernelGGL(k_colsum, dim3(1), dim3(1024), 0, t->st2, t->bpart[k], nwg_bwd, 64, 0, 64, G + L.cb[l]);
            HIP_TRY(hipEventRecord(t->ev_w[k], t->st2));
            used[k] = true;
            return 0;
        };
        if (int rc = wgrad()) return rc;
        if (l == 0) break;
        ConvArgs a{};
        a.in = dz;
        a.w = t->wd[l];
        a.out = t->M[l - 1];
        a.part = t->part;
        a.act = t->A[l - 1];
        a.zprev = t->Z[l - 1];
        a.mean = t->mean[l - 1];
        a.invstd = t->invstd[l - 1];
        a.skip = (l % 2 == 1) ? t->M[l + 1] : nullptr;  // first conv of a block: add the block-output gradient
        a.chunks = 4;
        a.B = B;
        launch_conv<CONV_DGRAD>(4, rg, conv_grid, st, a);
        nwg_part = nwg_conv;
    }
    HIP_TRY(hipEventRecord(t->ev_done, t->st2));
    HIP_TRY(hipStreamWaitEvent(st, t->ev_done, 0));  // every gradient is in G before SGD / all-reduce
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int oaz_trainer_backward(oaz_trainer* t, int b) {
    if (!t) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    if (!t->samples || b < 0 || b >= t->n_batches) return oaz_set_err(OAZ_ERR_STATE, "trainer: batch %d not uploaded", b);
    OAZ_ON_DEVICE(t->device);
    return backward(t, b);
}

extern "C" int oaz_trainer_grads(oaz_trainer* t, float** dev, size_t* n) {
    if (!t || !dev || !n) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    *dev = t->G;
    *n = t->nparam;
    return 0;
}

extern "C" int oaz_trainer_get_grads(oaz_trainer* t, float* host, size_t n) {
    if (!t || !host || n != t->nparam) return oaz_set_err(OAZ_ERR_ARG, "trainer: need %zu floats", t ? t->nparam : 0);
    OAZ_ON_DEVICE(t->device);
    HIP_TRY(hipMemcpyAsync(host, t->G, n * sizeof(float), hipMemcpyDeviceToHost, t->st));
    HIP_TRY(hipStreamSynchronize(t->st));
    return 0;
}

static int apply(oaz_trainer* t, float scale) {
    const long long n = (long long)t->nparam;
    ConvTab tab{};
    tab.n = t->nconv;
    for (int l = 0; l < t->nconv; ++l) {
        tab.off[l] = (int)t->L.cw[l];
        tab.cin[l] = l == 0 ? kIn : kC;
        tab.wf[l] = reinterpret_cast<float*>(t->wf[l]);
        tab.wd[l] = reinterpret_cast<float*>(t->wd[l]);
    }
    hipLaunchKernelGGL(k_sgd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, t->st, t->P, t->G, t->MOM, t->mask, n,
                       (float)t->cfg.learning_rate, (float)t->cfg.momentum, (float)t->cfg.weight_decay, scale, tab);
    HIP_TRY(hipGetLastError());
    return 0;
}

// BN running statistics <-> one contiguous range (data-parallel epoch-end average over ranks).
// Segments: per conv layer running_mean[64] running_var[64] (adjacent in the canonical blob), then
// the value head's (1 + 1) and the policy head's (2 + 2).
struct BnSegs {
    int n;
    int off[kMaxConv + 2], len[kMaxConv + 2];
};
static BnSegs bn_segs(const oaz_trainer* t) {
    BnSegs s{};
    for (int l = 0; l < t->nconv; ++l) {
        s.off[s.n] = (int)t->L.brm[l];
        s.len[s.n++] = 2 * kC;
    }
    s.off[s.n] = t->L.h.vrm;
    s.len[s.n++] = 2;
    s.off[s.n] = t->L.h.prm;
    s.len[s.n++] = 4;
    return s;
}
__global__ void k_bn_stats_io(float* P, float* buf, BnSegs s, int unpack, float scale) {
    int base = 0;
    for (int k = 0; k < s.n; ++k) {
        for (int i = threadIdx.x; i < s.len[k]; i += blockDim.x) {
            if (unpack) P[s.off[k] + i] = scale * buf[base + i];
            else buf[base + i] = P[s.off[k] + i];
        }
        base += s.len[k];
    }
}

extern "C" size_t oaz_trainer_bn_stats_count(int blocks) { return (size_t)(1 + 2 * blocks) * 2 * kC + 2 + 4; }

extern "C" int oaz_trainer_bn_stats_pack(oaz_trainer* t, float* dev_out) {
    if (!t || !dev_out) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    OAZ_ON_DEVICE(t->device);
    hipLaunchKernelGGL(k_bn_stats_io, dim3(1), dim3(256), 0, t->st, t->P, dev_out, bn_segs(t), 0, 1.0f);
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int oaz_trainer_bn_stats_unpack(oaz_trainer* t, const float* dev_in, float scale) {
    if (!t || !dev_in) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    OAZ_ON_DEVICE(t->device);
    hipLaunchKernelGGL(k_bn_stats_io, dim3(1), dim3(256), 0, t->st, t->P, const_cast<float*>(dev_in), bn_segs(t), 1,
                       scale);
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int oaz_trainer_apply(oaz_trainer* t, float grad_scale) {
    if (!t) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    OAZ_ON_DEVICE(t->device);
    return apply(t, grad_scale);
}

// One SGD step captured as a hipGraph (both streams; the batch number advances on the device),
// rebuilt when the batch size, stream or buffers change. Opt-in (OAZ_TRAIN_GRAPH=1).
static int ensure_graph(oaz_trainer* t) {
    const void* key[3] = {t->samples, t->idx, t->st};
    if (t->graph_exec && t->graph_batch == t->batch && !memcmp(key, t->graph_key, sizeof(key))) return 0;
    if (t->graph_exec) (void)hipGraphExecDestroy(t->graph_exec);
    if (t->graph) (void)hipGraphDestroy(t->graph);
    t->graph_exec = nullptr;
    t->graph = nullptr;
    HIP_TRY(hipStreamBeginCapture(t->st, hipStreamCaptureModeThreadLocal));
    int rc = backward(t, -1);
    if (!rc) rc = apply(t, 1.0f);
    if (!rc) hipLaunchKernelGGL(k_set_batch, dim3(1), dim3(64), 0, t->st, t->cur, 1, 1);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(t->st, &g);
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess) return oaz_set_err(OAZ_ERR_HIP, "trainer: graph capture: %s", hipGetErrorString(e));
    t->graph = g;
    HIP_TRY(hipGraphInstantiate(&t->graph_exec, g, nullptr, nullptr, 0));
    t->graph_batch = t->batch;
    memcpy(t->graph_key, key, sizeof(key));
    return 0;
}

extern "C" int oaz_trainer_train(oaz_trainer* t, int first, int count) {
    if (!t) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    if (!t->samples || first < 0 || count < 0 || first + count > t->n_batches)
        return oaz_set_err(OAZ_ERR_STATE, "trainer: batches [%d, %d) not uploaded", first, first + count);
    OAZ_ON_DEVICE(t->device);
    if (count == 0) return 0;
    // Plain stream launches by default: on this stack replaying the captured step (~65 kernels on
    // two streams) measured slower (1.06 vs 0.87 ms at batch 512, 5 blocks); OAZ_TRAIN_GRAPH=1
    // selects the graph path.
#if OAZ_AB
    const bool graph = getenv("OAZ_TRAIN_GRAPH") != nullptr;
#else
    const bool graph = false;
#endif
    if (!graph) {
        for (int b = first; b < first + count; ++b) {
            if (int rc = backward(t, b)) return rc;
            if (int rc = apply(t, 1.0f)) return rc;
        }
        return 0;
    }
    if (int rc = ensure_graph(t)) return rc;
    hipLaunchKernelGGL(k_set_batch, dim3(1), dim3(64), 0, t->st, t->cur, first, 0);
    HIP_TRY(hipGetLastError());
    for (int b = 0; b < count; ++b) HIP_TRY(hipGraphLaunch(t->graph_exec, t->st));
    return 0;
}

extern "C" int oaz_trainer_losses(oaz_trainer* t, double out[3]) {
    if (!t || !out) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    OAZ_ON_DEVICE(t->device);
    HIP_TRY(hipMemcpyAsync(out, t->loss_acc, 3 * sizeof(double), hipMemcpyDeviceToHost, t->st));
    HIP_TRY(hipMemsetAsync(t->loss_acc, 0, 3 * sizeof(double), t->st));
    HIP_TRY(hipStreamSynchronize(t->st));
    return 0;
}

extern "C" int oaz_trainer_sync(oaz_trainer* t) {
    if (!t) return oaz_set_err(OAZ_ERR_ARG, "trainer: null");
    OAZ_ON_DEVICE(t->device);
    HIP_TRY(hipStreamSynchronize(t->st));
    return 0;
}
