// oaz_nn.hip — ConvResNet policy-value forward (alphazero-training/src/net.rs:101-232), fused.
//
// One wavefront evaluates SPW positions end to end: encoder -> conv3x3(21->64) -> blocks x
// [conv3x3 -> relu -> conv3x3 -> +skip -> relu] -> value head -> policy head + softmax.
//   * 3x3 convs are implicit GEMMs on v_mfma_f32_32x32x2_f32 (exact f32 MFMA, no xf32 on
//     gfx950): M = one position's 25 squares padded to 32 rows, N = 64 output channels
//     (two 32-column tiles), K = 9 taps x Cin. A rows are gathered from the LDS activation
//     image through a per-lane neighbour index (off-board taps read a zero row); B fragments
//     are pre-packed on the host so each k-group is one coalesced 1 KiB dwordx4 load.
//   * BN (eval mode) is folded into the conv weights/bias on the host.
//   * activations never leave LDS (7 KB per position); the skip connection lives in
//     registers, so one LDS image per position suffices and convs write in place.
//   * the first layer never materialises the 21 planes: A values are computed from the
//     24-byte compact state (common.rs:26-80 semantics).
#include <hip/hip_runtime.h>

#include "oaz_device.h"
#include "oaz_kernels.h"

namespace oaz {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kCh = 64;
constexpr int kRS = 68;                      // LDS row stride (floats): 64 + 4 pad, no bank conflicts
constexpr int kRows = 26;                    // 25 squares + zero row
constexpr int kSampleFloats = kRows * kRS;   // 1768 floats = 7072 B
constexpr int kInitS = 12;                   // first layer: Cin 21 padded to 24, k-steps per tap per half
constexpr int kInitG = kInitS / 4;           // dwordx4 groups per tap
constexpr int kConvS = 32;                   // 64-channel layers: k-steps per tap per half
constexpr int kConvG = kConvS / 4;

// Packed blob layout (floats), built by pack_weights() in oaz_engine.cpp:
//   [init W: 9*3*2*64*4][init b: 64]
//   blocks x 2 x [W: 9*8*2*64*4][b: 64]
//   value:  wv[64] bv[1] pad[3] l1w[64*25] l1b[64] l2w[64] l2b[1] pad[3]
//   policy: wp[2*64] bp[2] pad[2] plw[50*50] plb[50] pad[2]
constexpr size_t kInitW = 9 * kInitG * 2 * 64 * 4;
constexpr size_t kConvW = 9 * kConvG * 2 * 64 * 4;
constexpr size_t kValueF = 64 + 4 + 64 * 25 + 64 + 64 + 4;
constexpr size_t kPolicyF = 128 + 4 + 2500 + 52;

size_t nn_packed_floats(int blocks) {
    return kInitW + kCh + (size_t)blocks * 2 * (kConvW + kCh) + kValueF + kPolicyF;
}

__device__ __forceinline__ int nbr_index(int i, int t) {
    // square i (row-major 5x5) shifted by tap t = (dy, dx) in {-1,0,1}^2; 25 = off board
    if (i >= 25) return 25;
    const int r = i / 5 + t / 3 - 1, c = i % 5 + t % 3 - 1;
    return (r >= 0 && r < 5 && c >= 0 && c < 5) ? r * 5 + c : 25;
}

// Input plane `ci` (0..23, 21..23 zero padding) of state s at square sq (25 = off board).
__device__ __forceinline__ float plane_value(const oaz_state& s, int ci, int sq) {
    if (sq >= 25) return 0.0f;
    const int color = s.to_move & 1;
    if (ci < 4) {
        const uint32_t src = ci == 0 ? s.pawns[0] : ci == 1 ? s.kings[0] : ci == 2 ? s.pawns[1] : s.kings[1];
        return (src & sq_bit(sq)) ? 1.0f : 0.0f;
    }
    if (ci < 20) {  // the mover's two cards (static indices: no local-array promotion)
        const int c0 = (color ? s.cards[2] : s.cards[0]) & 15, c1 = (color ? s.cards[3] : s.cards[1]) & 15;
        return (c0 == ci - 4 || c1 == ci - 4) ? 1.0f : 0.0f;
    }
    if (ci == 20) return color ? 1.0f : 0.0f;
    return 0.0f;
}

template <int SPW>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[SPW][2]) {
#pragma unroll
    for (int sp = 0; sp < SPW; ++sp) {
        acc[sp][0] = f32x16{};
        acc[sp][1] = f32x16{};
    }
}

// acc += conv3x3(act) over 64 input channels; ci = h*32 + 4*grp + q.
template <int SPW>
__device__ __forceinline__ void conv64(f32x16 (&acc)[SPW][2], const float* act, const float4* W,
                                       int lane) {
    const int i = lane & 31, h = lane >> 5;
    float4 b0 = W[0 * 64 + lane], b1 = W[1 * 64 + lane];
    for (int t = 0; t < 9; ++t) {
        const int row = nbr_index(i, t);
        const float* arow = act + row * kRS + h * 32;
#pragma unroll 2
        for (int grp = 0; grp < kConvG; ++grp) {
            const int gi = t * kConvG + grp;
            float4 n0 = b0, n1 = b1;
            if (gi + 1 < 9 * kConvG) {
                n0 = W[((gi + 1) * 2 + 0) * 64 + lane];
                n1 = W[((gi + 1) * 2 + 1) * 64 + lane];
            }
            float4 a[SPW];
#pragma unroll
            for (int sp = 0; sp < SPW; ++sp)
                a[sp] = *reinterpret_cast<const float4*>(arow + sp * kSampleFloats + 4 * grp);
#pragma unroll
            for (int sp = 0; sp < SPW; ++sp) {
                acc[sp][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].x, b0.x, acc[sp][0], 0, 0, 0);
                acc[sp][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].x, b1.x, acc[sp][1], 0, 0, 0);
            }
#pragma unroll
            for (int sp = 0; sp < SPW; ++sp) {
                acc[sp][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].y, b0.y, acc[sp][0], 0, 0, 0);
                acc[sp][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].y, b1.y, acc[sp][1], 0, 0, 0);
            }
#pragma unroll
            for (int sp = 0; sp < SPW; ++sp) {
                acc[sp][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].z, b0.z, acc[sp][0], 0, 0, 0);
                acc[sp][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].z, b1.z, acc[sp][1], 0, 0, 0);
            }
#pragma unroll
            for (int sp = 0; sp < SPW; ++sp) {
                acc[sp][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].w, b0.w, acc[sp][0], 0, 0, 0);
                acc[sp][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sp].w, b1.w, acc[sp][1], 0, 0, 0);
            }
            b0 = n0;
            b1 = n1;
        }
    }
}

// C/D layout of v_mfma_f32_32x32x2f32: reg r of lane l holds row (r&3)+8*(r>>2)+4*(l>>5),
// column l&31. Rows are squares (>=25: padding), columns output channels.
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

template <int SPW>
__device__ __forceinline__ void epilogue(const f32x16 (&acc)[SPW][2], float* act, const float* bias,
                                         const f32x16 (*skip)[2], int lane) {
    const int i = lane & 31;
    const float bb0 = bias[i], bb1 = bias[32 + i];
#pragma unroll
    for (int sp = 0; sp < SPW; ++sp) {
        float* a = act + sp * kSampleFloats;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = acc_row(r, lane);
            if (row < 25) {
                float v0 = acc[sp][0][r] + bb0;
                float v1 = acc[sp][1][r] + bb1;
                if (skip) {
                    v0 += skip[sp][0][r];
                    v1 += skip[sp][1][r];
                }
                a[row * kRS + i] = v0 > 0.0f ? v0 : 0.0f;
                a[row * kRS + 32 + i] = v1 > 0.0f ? v1 : 0.0f;
            }
        }
    }
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

template <int SPW, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_nn_forward(const oaz_state* __restrict__ states, int B,
                                                         const float* __restrict__ blob, int blocks,
                                                         float* __restrict__ policy,
                                                         float* __restrict__ value) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = lane & 31, h = lane >> 5;
    float* act = smem + (size_t)wave * SPW * kSampleFloats;
    const int b0 = (blockIdx.x * WPB + wave) * SPW;
    if (b0 >= B) return;  // whole wave idle (no block-level barriers in this kernel)

    oaz_state st[SPW];
#pragma unroll
    for (int sp = 0; sp < SPW; ++sp) {
        const int b = b0 + sp < B ? b0 + sp : b0;
        st[sp] = states[b];
        act[sp * kSampleFloats + 25 * kRS + lane] = 0.0f;  // zero row (64 channels)
    }

    // ---- initial block: conv3x3(21->64)+BN+ReLU (net.rs:119-136) ----
    f32x16 acc[SPW][2];
    zero_acc<SPW>(acc);
    const float* p = blob;
    {
        const float4* W = reinterpret_cast<const float4*>(p);
        for (int t = 0; t < 9; ++t) {
            const int sq = nbr_index(i, t);
#pragma unroll
            for (int grp = 0; grp < kInitG; ++grp) {
                const float4 w0 = W[((t * kInitG + grp) * 2 + 0) * 64 + lane];
                const float4 w1 = W[((t * kInitG + grp) * 2 + 1) * 64 + lane];
                const float wb0[4] = {w0.x, w0.y, w0.z, w0.w};
                const float wb1[4] = {w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int ci = h * kInitS + 4 * grp + q;
#pragma unroll
                    for (int sp = 0; sp < SPW; ++sp) {
                        const float av = plane_value(st[sp], ci, sq);
                        acc[sp][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wb0[q], acc[sp][0], 0, 0, 0);
                        acc[sp][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wb1[q], acc[sp][1], 0, 0, 0);
                    }
                }
            }
        }
        p += kInitW;
        epilogue<SPW>(acc, act, p, nullptr, lane);
        p += kCh;
    }

    // ---- residual tower (net.rs:39-66, 138-147) ----
    for (int blk = 0; blk < blocks; ++blk) {
        f32x16 skip[SPW][2];
#pragma unroll
        for (int sp = 0; sp < SPW; ++sp)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = acc_row(r, lane);
                const float* a = act + sp * kSampleFloats + (row < 25 ? row : 25) * kRS;
                skip[sp][0][r] = a[i];
                skip[sp][1][r] = a[32 + i];
            }
        zero_acc<SPW>(acc);
        conv64<SPW>(acc, act, reinterpret_cast<const float4*>(p), lane);
        p += kConvW;
        epilogue<SPW>(acc, act, p, nullptr, lane);
        p += kCh;
        zero_acc<SPW>(acc);
        conv64<SPW>(acc, act, reinterpret_cast<const float4*>(p), lane);
        p += kConvW;
        epilogue<SPW>(acc, act, p, skip, lane);
        p += kCh;
    }

    // ---- heads (net.rs:152-213), per position ----
    const float* vw = p;
    const float vb = p[64];
    const float* l1w = p + 68;
    const float* l1b = l1w + 64 * 25;
    const float* l2w = l1b + 64;
    const float l2b = l2w[64];
    const float* pp = p + kValueF;
    const float* pw = pp;
    const float pb0 = pp[128], pb1 = pp[129];
    const float* plw = pp + 132;
    const float* plb = plw + 2500;
    for (int sp = 0; sp < SPW; ++sp) {
        float* a = act + sp * kSampleFloats;
        // 1x1 convs (value 64->1, policy 64->2) with folded BN, ReLU; lane = square
        float v1 = 0.0f, c0 = 0.0f, c1 = 0.0f;
        if (lane < 25) {
            float sv = vb, s0 = pb0, s1 = pb1;
            const float* row = a + lane * kRS;
            for (int c = 0; c < kCh; c += 4) {
                const float4 x = *reinterpret_cast<const float4*>(row + c);
                sv += vw[c] * x.x + vw[c + 1] * x.y + vw[c + 2] * x.z + vw[c + 3] * x.w;
                s0 += pw[c] * x.x + pw[c + 1] * x.y + pw[c + 2] * x.z + pw[c + 3] * x.w;
                s1 += pw[64 + c] * x.x + pw[65 + c] * x.y + pw[66 + c] * x.z + pw[67 + c] * x.w;
            }
            v1 = sv > 0.0f ? sv : 0.0f;
            c0 = s0 > 0.0f ? s0 : 0.0f;
            c1 = s1 > 0.0f ? s1 : 0.0f;
        }
        // stage the flattened head inputs in the (now free) first rows of the image
        if (lane < 25) {
            a[lane] = v1;          // value features [25]
            a[32 + lane] = c0;     // policy features [o*25+p] at 32..81
            a[57 + lane] = c1;
        }
        // value: linear 25->64, ReLU, linear 64->1, tanh
        float hj = l1b[lane];
        for (int q = 0; q < 25; ++q) hj += l1w[lane * 25 + q] * a[q];
        hj = hj > 0.0f ? hj : 0.0f;
        const float vsum = wave_sum_f(l2w[lane] * hj);
        // policy: linear 50->50, softmax over all 50 (net.rs:205-212)
        float lg = -INFINITY;
        if (lane < 50) {
            lg = plb[lane];
            for (int f = 0; f < 50; ++f) lg += plw[lane * 50 + f] * a[32 + f];
        }
        const float mx = wave_max_f(lg);
        const float e = lane < 50 ? expf(lg - mx) : 0.0f;
        const float den = wave_sum_f(e);
        const int b = b0 + sp;
        if (b < B) {
            if (lane < 50) policy[(size_t)b * 50 + lane] = e / den;
            if (lane == 0) value[b] = tanhf(vsum + l2b);
        }
    }
}

// ===========================================================================================
// v2: square-major tiles, off-board taps skipped.
//   A workgroup evaluates 16 positions. Its 400 GEMM rows are ordered square-major
//   (row = square*16 + position), so M-tile m is "square m of all 16 positions". For tap t the
//   neighbour of square m is either on the board for the whole tile or off it for the whole
//   tile: off-board tiles are skipped instead of multiplied by a zero row — 169 of the 225
//   (tile, tap) products of a 5x5 board are computed, the dense GEMM's padding work is gone.
//   8 waves: wave w owns output channels 16*(w&3)..+15 and square group w>>2; the two groups
//   (13 and 12 squares) carry 85 and 84 on-board (square, tap) pairs, so the two waves that
//   share a SIMD are balanced. Two waves per SIMD (<= 256 VGPRs). Layers are separated by
//   workgroup barriers (every wave reads all input channels of its squares' neighbours).
// ===========================================================================================
namespace v2 {
constexpr int kSB = 16;                  // positions per workgroup (= rows per M-tile)
constexpr int kWaves = 8;
constexpr int kTPW = 13;                 // squares per wave group (group 1: 12)
// Row stride 72 floats and channel order ci = 16g + 4kq + q: the 16-lane groups of a
// ds_read_b128 (lanes = 16 consecutive rows x 4 channel quarters) hit 16 distinct 16-byte
// bank slots (row*18 + kq mod 16), so the A gathers are conflict-free.
constexpr int kRS2 = 72;
constexpr int kScratch = 128;            // per-wave head scratch (floats)
constexpr int kLdsFloats = kSB * 25 * kRS2 + kWaves * kScratch;  // 29824 floats = 119,296 B
constexpr size_t kW0 = 9 * 2 * 4 * 64 * 4;   // first layer, Cin padded 21 -> 32
constexpr size_t kW64 = 9 * 4 * 4 * 64 * 4;  // 64 -> 64
}  // namespace v2

// Square groups: 4 corners + 4 edges + 5 interior (85 on-board taps) | 8 edges + 4 interior (84).
__constant__ int8_t c_sq_order[25] = {0, 4, 20, 24, 1, 3, 21, 23, 6, 8, 12, 16, 18,
                                      2, 5, 10, 15, 9, 14, 19, 22, 7, 11, 13, 17};

typedef float f32x4 __attribute__((ext_vector_type(4)));

size_t nn2_packed_floats(int blocks) {
    return v2::kW0 + kCh + (size_t)blocks * 2 * (v2::kW64 + kCh) + kValueF + kPolicyF;
}

// acc[j] += conv3x3 over CIN = 16*G input channels for square sq[j] (j < ntiles).
// K order per tap: at k-step (g, q) lane group kq = lane>>4 supplies channel 16g + 4kq + q.
template <int G>
__device__ __forceinline__ void conv_sq(f32x4 (&acc)[v2::kTPW], const float* act, const float4* W,
                                        const int (&sq)[v2::kTPW], int lane, int nt, int ntiles) {
    const int i = lane & 15, kq = lane >> 4;
    const float* base = act + i * v2::kRS2 + 4 * kq;
    for (int t = 0; t < 9; ++t) {
        int off[v2::kTPW];  // wave-uniform: row offset of the neighbour square, -1 if off board
#pragma unroll
        for (int j = 0; j < v2::kTPW; ++j) {
            const int nb = nbr_index(sq[j], t);
            off[j] = (j < ntiles && nb < 25) ? nb * v2::kSB * v2::kRS2 : -1;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float4 b = W[((t * G + g) * 4 + nt) * 64 + lane];
#pragma unroll
            for (int j = 0; j < v2::kTPW; ++j)
                if (off[j] >= 0) {
                    const float4 a = *reinterpret_cast<const float4*>(base + off[j] + 16 * g);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[j], 0, 0, 0);
                }
        }
    }
}

// C/D of v_mfma_f32_16x16x4_f32: reg r of lane l = (row (l>>4)*4 + r, col l&15) of the tile,
// i.e. position (l>>4)*4 + r at square sq[j]; LDS row = square*16 + position.
__device__ __forceinline__ void epilogue_sq(const f32x4 (&acc)[v2::kTPW], float* act, const float* bias,
                                            const f32x4* skip, const int (&sq)[v2::kTPW], int lane, int nt,
                                            int ntiles) {
    const int co = nt * 16 + (lane & 15);
    const float bb = bias[co];
#pragma unroll
    for (int j = 0; j < v2::kTPW; ++j)
        if (j < ntiles)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = sq[j] * v2::kSB + (lane >> 4) * 4 + r;
                float v = acc[j][r] + bb;
                if (skip) v += skip[j][r];
                act[row * v2::kRS2 + co] = v > 0.0f ? v : 0.0f;
            }
}

__device__ __forceinline__ void read_skip_sq(f32x4 (&skip)[v2::kTPW], const float* act, const int (&sq)[v2::kTPW],
                                             int lane, int nt, int ntiles) {
    const int co = nt * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < v2::kTPW; ++j)
        if (j < ntiles)
#pragma unroll
            for (int r = 0; r < 4; ++r) skip[j][r] = act[(sq[j] * v2::kSB + (lane >> 4) * 4 + r) * v2::kRS2 + co];
}

// value + policy heads (net.rs:152-213) for position `s` of the workgroup (one wave).
__device__ __forceinline__ void heads_sq(const float* act, float* scratch, int s, const float* p, int lane, int b,
                                         int B, float* policy, float* value) {
    const float* vw = p;
    const float vb = p[64];
    const float* l1w = p + 68;
    const float* l1b = l1w + 64 * 25;
    const float* l2w = l1b + 64;
    const float l2b = l2w[64];
    const float* pp = p + kValueF;
    const float pb0 = pp[128], pb1 = pp[129];
    const float* plw = pp + 132;
    const float* plb = plw + 2500;
    if (lane < 25) {  // 1x1 convs (value 64->1, policy 64->2) with folded BN, ReLU; lane = square
        float sv = vb, s0 = pb0, s1 = pb1;
        const float* row = act + (lane * v2::kSB + s) * v2::kRS2;
        for (int c = 0; c < kCh; c += 4) {
            const float4 x = *reinterpret_cast<const float4*>(row + c);
            sv += vw[c] * x.x + vw[c + 1] * x.y + vw[c + 2] * x.z + vw[c + 3] * x.w;
            s0 += pp[c] * x.x + pp[c + 1] * x.y + pp[c + 2] * x.z + pp[c + 3] * x.w;
            s1 += pp[64 + c] * x.x + pp[65 + c] * x.y + pp[66 + c] * x.z + pp[67 + c] * x.w;
        }
        scratch[lane] = sv > 0.0f ? sv : 0.0f;       // value features [25]
        scratch[32 + lane] = s0 > 0.0f ? s0 : 0.0f;  // policy features, flatten(1,-1) order
        scratch[57 + lane] = s1 > 0.0f ? s1 : 0.0f;
    }
    float hj = l1b[lane];
    for (int q = 0; q < 25; ++q) hj += l1w[lane * 25 + q] * scratch[q];
    hj = hj > 0.0f ? hj : 0.0f;
    const float vsum = wave_sum_f(l2w[lane] * hj);
    float lg = -INFINITY;
    if (lane < 50) {
        lg = plb[lane];
        for (int f = 0; f < 50; ++f) lg += plw[lane * 50 + f] * scratch[32 + f];
    }
    const float mx = wave_max_f(lg);
    const float e = lane < 50 ? expf(lg - mx) : 0.0f;
    const float den = wave_sum_f(e);
    if (b < B) {
        if (lane < 50) policy[(size_t)b * 50 + lane] = e / den;
        if (lane == 0) value[b] = tanhf(vsum + l2b);
    }
}

__global__ void __launch_bounds__(64 * v2::kWaves) k_nn_sq16(const oaz_state* __restrict__ states, int B,
                                                             const float* __restrict__ blob, int blocks,
                                                             float* __restrict__ policy,
                                                             float* __restrict__ value) {
    __shared__ __attribute__((aligned(16))) float act[v2::kLdsFloats];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nt = wave & 3, grp = wave >> 2;
    const int ntiles = grp == 0 ? v2::kTPW : 25 - v2::kTPW;
    int sq[v2::kTPW];
#pragma unroll
    for (int j = 0; j < v2::kTPW; ++j) sq[j] = (j < ntiles) ? c_sq_order[grp * v2::kTPW + j] : 0;
    const int b0 = blockIdx.x * v2::kSB;

    // encoder (common.rs:26-80): 21 planes, zero-padded to 32 channels, from the 24-byte state
    if (tid < v2::kSB * 25) {
        const int sqr = tid / v2::kSB, pos = tid - v2::kSB * sqr;
        const int b = b0 + pos < B ? b0 + pos : b0;
        const oaz_state st = states[b];
        float* row = act + tid * v2::kRS2;
#pragma unroll
        for (int c = 0; c < 32; c += 4) {
            float4 v;
            v.x = plane_value(st, c, sqr);
            v.y = plane_value(st, c + 1, sqr);
            v.z = plane_value(st, c + 2, sqr);
            v.w = plane_value(st, c + 3, sqr);
            *reinterpret_cast<float4*>(row + c) = v;
        }
    }
    __syncthreads();

    f32x4 acc[v2::kTPW];
    f32x4 skip[v2::kTPW];
    const float* p = blob;
#pragma unroll
    for (int j = 0; j < v2::kTPW; ++j) acc[j] = f32x4{};
    conv_sq<2>(acc, act, reinterpret_cast<const float4*>(p), sq, lane, nt, ntiles);
    p += v2::kW0;
    __syncthreads();
    epilogue_sq(acc, act, p, nullptr, sq, lane, nt, ntiles);
    p += kCh;
    __syncthreads();

    for (int blk = 0; blk < blocks; ++blk) {
        read_skip_sq(skip, act, sq, lane, nt, ntiles);
#pragma unroll
        for (int j = 0; j < v2::kTPW; ++j) acc[j] = f32x4{};
        conv_sq<4>(acc, act, reinterpret_cast<const float4*>(p), sq, lane, nt, ntiles);
        p += v2::kW64;
        __syncthreads();
        epilogue_sq(acc, act, p, nullptr, sq, lane, nt, ntiles);
        p += kCh;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < v2::kTPW; ++j) acc[j] = f32x4{};
        conv_sq<4>(acc, act, reinterpret_cast<const float4*>(p), sq, lane, nt, ntiles);
        p += v2::kW64;
        __syncthreads();
        epilogue_sq(acc, act, p, skip, sq, lane, nt, ntiles);
        p += kCh;
        __syncthreads();
    }
    float* scratch = act + v2::kSB * 25 * v2::kRS2 + wave * v2::kScratch;
    for (int s = wave; s < v2::kSB; s += v2::kWaves) heads_sq(act, scratch, s, p, lane, b0 + s, B, policy, value);
}

constexpr int kSPW = 2;
constexpr int kWPB = 4;

hipError_t launch_nn_forward(const NNView& w, const oaz_state* s, int B, float* policy,
                             float* value, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    if (w.variant == 2) {
        const unsigned grid2 = (unsigned)((B + v2::kSB - 1) / v2::kSB);
        hipLaunchKernelGGL(k_nn_sq16, dim3(grid2), dim3(64 * v2::kWaves), 0, st, s, B, w.blob2, w.blocks, policy,
                           value);
        return hipGetLastError();
    }
    const int per_block = kSPW * kWPB;
    const unsigned grid = (unsigned)((B + per_block - 1) / per_block);
    const size_t lds = (size_t)kWPB * kSPW * kSampleFloats * sizeof(float);
    hipLaunchKernelGGL((k_nn_forward<kSPW, kWPB>), dim3(grid), dim3(64 * kWPB), lds, st, s, B,
                       w.blob, w.blocks, policy, value);
    return hipGetLastError();
}

}  // namespace oaz
