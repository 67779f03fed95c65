// oaz_nn.hip — ConvResNet policy-value forward (alphazero-training/src/net.rs:101-232), fused
// into one kernel: encoder -> conv3x3(21->64)+BN+ReLU -> blocks x [conv3x3+BN+ReLU ->
// conv3x3+BN -> +skip -> ReLU] -> value head (1x1 conv, MLP, tanh) -> policy head (1x1 conv,
// linear, softmax over 50). One kernel per oaz_config.precision:
//   k_nn_h3   OAZ_FP32_SPLIT16 (the benches' fp32 kernel): fp32 operands split into hi + lo fp16
//             terms, three products on v_mfma_f32_16x16x32_f16; fp16-range tiles recomputed in the
//             same launch with the k_nn_x6 body. With H3Cfg<1> the same structure in OAZ_BF16 (C5).
//   k_nn_x6   OAZ_FP32_SPLIT: an exact three-term bf16 split, six products on 16x16x32 bf16 MFMA.
//   k_nn_sq16 OAZ_FP32: exact fp32 products on v_mfma_f32_16x16x4_f32.
// DESIGN.md section 5 describes each; below, k_nn_sq16's geometry, which the others refine.
//
// Geometry (k_nn_sq16)
//   * A workgroup evaluates 16 positions. The 3x3 convs are implicit GEMMs whose 400 rows are ordered
//     SQUARE-MAJOR (row = square*16 + position): an M-tile is one board square of all 16
//     positions. For a tap, a tile's neighbour square is on the board for the whole tile or off
//     it for the whole tile, so off-board products are skipped instead of multiplied by zero
//     padding: 169 of the 225 (square, tap) products of a 5x5 board are computed.
//   * 8 waves: wave w owns output channels 16*(w&3)..+15 and square group w>>2. The two groups
//     (4 corners + 4 edges + 5 interior | 8 edges + 4 interior) carry 85 and 84 on-board
//     (square, tap) pairs, and waves w, w+4 share a SIMD, so SIMDs are balanced.
//   * Activations stay in LDS for the whole tower (row stride 72 floats, channel order
//     16g + 4*(lane>>4) + q: the ds_read_b128 A gathers are bank-conflict free); the residual
//     skip is kept in registers; each conv writes its output in place between barriers.
//   * BN (eval) is folded on the host; B fragments are packed so that each k-group is one
//     coalesced 1 KiB dwordx4 load per wave.
//   * First layer: of the 21 input planes (common.rs:26-80) only the 4 bitboards vary across
//     the board; the 16 card planes and the side-to-move plane are constant over all squares,
//     so their contribution is the host-precomputed table T[square][card][channel] (sum of the
//     folded weights over the on-board taps). The 21 planes are never materialised.
#include <hip/hip_runtime.h>

#include <utility>

#include "oaz_device.h"
#include "oaz_kernels.h"

namespace oaz {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace nn {
constexpr int kCh = 64;
constexpr int kSB = 16;      // positions per workgroup (= rows per M-tile)
constexpr int kWaves = 8;
constexpr int kTPW = 13;     // squares per wave group (group 1: 12)
constexpr int kRS = 72;      // LDS row stride (floats)
constexpr int kScratch = 128;  // per-wave head scratch (floats)
constexpr int kLdsFloats = kSB * 25 * kRS + kWaves * kScratch;  // 29824 floats = 119,296 B
// Packed blob (floats), built by pack_weights() in oaz_engine.cpp:
//   [L1 B: 9 taps x 4 N-tiles x 64 lanes][L1 bias 64][L1 table: 25 squares x 17 x 64]
//   blocks x 2 x [W: 9 taps x 4 groups x 4 N-tiles x 64 lanes x 4][bias 64]
//   value head:  wv[64] bv pad[3] l1w[25][64] (transposed) l1b[64] l2w[64] l2b pad[3]
//   policy head: wp[2*64] bp[2] pad[2] plw[50 in][50 out] (transposed) plb[50] pad[2]
constexpr size_t kL1B = 9 * 4 * 64;
constexpr size_t kL1Table = 25 * 17 * kCh;
constexpr size_t kW64 = 9 * 4 * 4 * 64 * 4;
constexpr size_t kValueF = 64 + 4 + 64 * 25 + 64 + 64 + 4;
constexpr size_t kPolicyF = 128 + 4 + 2500 + 52;

// OAZ_BF16 (k_nn_h3 in bf16 mode): 64->64 conv B fragments are bf16 [9 taps][2 K-halves][4 N-tiles]
// [64 lanes][8], stored in the float blob as 9*2*4*64*4 floats
constexpr size_t kW64h = 9 * 2 * 4 * 64 * 4;

}  // namespace nn

// Rows of this workgroup: [b0, b0 + kSB) below `end`; row loads are clamped to `cap` rows. Plain
// tiles cover [0, B); over compacted leaves (TileMap, oaz_kernels.h) workgroup i takes tile i / nb of
// bucket i % nb, and a tile past its bucket's count exits after its first loads.
struct TileSpan {
    int b0, end, cap;
};
__device__ __forceinline__ TileSpan tile_span(const TileMap& tm, int B) {
    if (!tm.bcnt) return TileSpan{(int)blockIdx.x * nn::kSB, B, B};
    const int b = (int)blockIdx.x % tm.nb, t = (int)blockIdx.x / tm.nb, base = b << kBucketShift;
    return TileSpan{base + t * nn::kSB, base + (int)tm.bcnt[b], tm.cap};
}

// fp32 split variant (OAZ_FP32_SPLIT): 64->64 conv B fragments are [9 taps][2 K-halves][3 pieces]
// [4 N-tiles][64 lanes] bf16x8 (the exact 3-term bf16 split of each folded fp32 weight).
namespace x6 {
constexpr int kRowB = 384;                  // LDS row: 3 pieces x 64 channels x bf16, no padding
constexpr int kImageB = nn::kSB * 25 * kRowB;  // 153,600 B
constexpr int kLdsFloats = kImageB / 4 + nn::kWaves * nn::kScratch;  // 39,424 floats = 157,696 B
constexpr size_t kW = 9 * 2 * 3 * 4 * 64 * 4;
constexpr size_t kHeadB = 2 * 3 * 64 * 4;  // head 1x1 convs: [K-half][piece][lane] bf16x8 (after the heads)
}  // namespace x6

// fp16 split variant (OAZ_FP32_SPLIT16): 64->64 conv B fragments are [9 taps][2 K-halves][2 pieces]
// [4 N-tiles][64 lanes] f16x8 of the per-output-channel scaled weights, then bias[64] and the
// inverse scales[64]; the head 1x1 convs [K-half][piece][lane] f16x8 + 4 inverse column scales.
namespace h3 {
constexpr int kRowB = 128;                     // LDS row of one piece plane: 64 channels x f16
constexpr int kPlaneB = nn::kSB * 25 * kRowB;  // 51,200 B per piece plane
constexpr int kImageB = 2 * kPlaneB;           // 102,400 B
constexpr int kLdsFloats = kImageB / 4 + nn::kWaves * nn::kScratch;  // 26,624 floats = 106,496 B
constexpr size_t kW = 9 * 2 * 2 * 4 * 64 * 4;
constexpr size_t kHeadB = 2 * 2 * 64 * 4 + 4;
// first layer on fp16 MFMA (k_nn_h3, TR): K block 0 [piece][N-tile][lane] f16x8 (bitboard taps 0-7 of
// plane q = lane >> 4, square-independent), K block 1 [square][piece][N-tile][lane] f16x8 (tap 8 of
// plane q, then the 17 constant planes' table T[square]), all scaled by s = 2^k per output channel;
// then 1/s[64]. The 0/1 B operands are built in-kernel (lut: LDS table of the 8-tap bit patterns).
constexpr size_t kL1Frag = 2 * 4 * 64 * 4;            // one K block: 2 pieces x 4 N-tiles x 64 lanes x f16x8
constexpr size_t kL1C = 26 * kL1Frag + nn::kCh;
constexpr int kLutB = 256 * 16;                       // 256 patterns x f16x8
constexpr int kLutOff = kLdsFloats * 4;               // after the image + scratch (the fallback's LDS)
}  // namespace h3

size_t nn_packed_floats(int blocks, int precision) {
    if (precision == OAZ_FP32_SPLIT16)
        return nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh) + nn::kValueF +
               nn::kPolicyF + h3::kHeadB + h3::kL1C;
    const size_t w = precision == OAZ_BF16 ? nn::kW64h : precision == OAZ_FP32_SPLIT ? x6::kW : nn::kW64;
    return nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (w + nn::kCh) + nn::kValueF + nn::kPolicyF +
           (precision == OAZ_FP32_SPLIT ? x6::kHeadB : 0) + (precision == OAZ_BF16 ? 2 * 64 * 4 + h3::kL1C : 0);
}

// Square groups: 4 corners + 4 edges + 5 interior (85 on-board taps) | 8 edges + 4 interior (84).
__constant__ int8_t c_sq_order[25] = {0, 4, 20, 24, 1, 3, 21, 23, 6, 8, 12, 16, 18,
                                      2, 5, 10, 15, 9, 14, 19, 22, 7, 11, 13, 17};

__device__ __forceinline__ int nbr_index(int sq, int t) {
    // square sq (row-major 5x5) shifted by tap t = (dy, dx) in {-1,0,1}^2; 25 = off board
    const int r = sq / 5 + t / 3 - 1, c = sq % 5 + t % 3 - 1;
    return (r >= 0 && r < 5 && c >= 0 && c < 5) ? r * 5 + c : 25;
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

// First layer, bitboard part: acc[j] += sum over on-board taps of bit(plane kq, neighbour) *
// W[co][kq][tap] — one v_mfma_f32_16x16x4_f32 per (square, tap), K = the 4 bitboards.
__device__ __forceinline__ void conv_l1(f32x4 (&acc)[nn::kTPW], uint32_t bb, const float* W,
                                        const int (&sq)[nn::kTPW], int lane, int nt, int ntiles) {
    for (int t = 0; t < 9; ++t) {
        const float b = W[(t * 4 + nt) * 64 + lane];
#pragma unroll
        for (int j = 0; j < nn::kTPW; ++j) {
            const int nb = nbr_index(sq[j], t);
            if (j < ntiles && nb < 25) {
                const float a = (float)((bb >> (31 - nb)) & 1u);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
            }
        }
    }
}

// acc[j] += conv3x3 over 64 input channels for square sq[j] (j < ntiles).
// K order per tap: at k-step (g, q) lane group kq = lane>>4 supplies channel 16g + 4kq + q.
__device__ __forceinline__ void conv64(f32x4 (&acc)[nn::kTPW], const float* act, const float4* W,
                                       const int (&sq)[nn::kTPW], int lane, int nt, int ntiles) {
    const int i = lane & 15, kq = lane >> 4;
    const float* base = act + i * nn::kRS + 4 * kq;
    for (int t = 0; t < 9; ++t) {
        // Wave-uniform (scalar) neighbour offsets and on-board mask: the skip test becomes a scalar
        // branch, and every A fragment of a k-group is requested before the first MFMA so the LDS
        // latency hides behind the MFMAs of the earlier squares. Off-board squares load a harmless
        // row (their own square) and skip their MFMAs.
        int off[nn::kTPW];
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < nn::kTPW; ++j) {
            const int nb = nbr_index(sq[j], t);
            const bool ok = j < ntiles && nb < 25;
            off[j] = __builtin_amdgcn_readfirstlane((ok ? nb : sq[j]) * nn::kSB * nn::kRS);
            vm |= (ok ? 1u : 0u) << j;
        }
        vm = __builtin_amdgcn_readfirstlane(vm);
        float4 b = W[((t * 4 + 0) * 4 + nt) * 64 + lane];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 bn = W[((t * 4 + (g < 3 ? g + 1 : g)) * 4 + nt) * 64 + lane];  // next k-group's B
            constexpr int kH = (nn::kTPW + 1) / 2;  // two batches of A fragments (register budget)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float4 a[kH];
#pragma unroll
                for (int q = 0; q < kH; ++q) {
                    const int j = h * kH + q;
                    if (j < nn::kTPW) a[q] = *reinterpret_cast<const float4*>(base + off[j] + 16 * g);
                }
#pragma unroll
                for (int q = 0; q < kH; ++q) {
                    const int j = h * kH + q;
                    if (j < nn::kTPW && (vm & (1u << j))) {
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].x, b.x, acc[j], 0, 0, 0);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].y, b.y, acc[j], 0, 0, 0);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].z, b.z, acc[j], 0, 0, 0);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].w, b.w, acc[j], 0, 0, 0);
                    }
                }
            }
            b = bn;
        }
    }
}

// First layer, constant planes: the mover's two card planes and the blue-to-move plane are
// constant over the board, so per square their contribution is sum_c onehot[pos][c] * T[sq][c][co]
// with T the host table (folded weights summed over the on-board taps). That is a K = 17 (padded
// to 20) GEMM per square: 5 v_mfma_f32_16x16x4_f32 whose A operand (0/1) is built from the
// position's cards in registers and whose B operand is read from the table, all loads independent.
__device__ __forceinline__ void conv_l1_const(f32x4 (&acc)[nn::kTPW], const float* table, int cinfo,
                                              const int (&sq)[nn::kTPW], int lane, int nt, int ntiles) {
    const int kq = lane >> 4, co = nt * 16 + (lane & 15);
    const int c0 = cinfo & 15, c1 = (cinfo >> 4) & 15, blue = (cinfo >> 8) & 1;
    float a[5];
#pragma unroll
    for (int st = 0; st < 5; ++st) {
        const int k = 4 * st + kq;
        a[st] = k < 16 ? ((k == c0 || k == c1) ? 1.0f : 0.0f) : (k == 16 ? (float)blue : 0.0f);
    }
#pragma unroll
    for (int j = 0; j < nn::kTPW; ++j)
        if (j < ntiles) {
            const float* ts = table + (size_t)sq[j] * 17 * nn::kCh + co;
            float b[5];
#pragma unroll
            for (int st = 0; st < 5; ++st) {
                const int k = 4 * st + kq;
                b[st] = k < 17 ? ts[k * nn::kCh] : 0.0f;
            }
#pragma unroll
            for (int st = 0; st < 5; ++st) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[st], b[st], acc[j], 0, 0, 0);
        }
}

// C/D of v_mfma_f32_16x16x4_f32: reg r of lane l = (row (l>>4)*4 + r, col l&15) of the tile,
// i.e. position (l>>4)*4 + r at square sq[j]; LDS row = square*16 + position.
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[nn::kTPW], float* act, const float* bias, const f32x4* skip,
                                         const int (&sq)[nn::kTPW], int lane, int nt, int ntiles) {
    const int co = nt * 16 + (lane & 15);
    const float bb = bias[co];
#pragma unroll
    for (int j = 0; j < nn::kTPW; ++j)
        if (j < ntiles)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = sq[j] * nn::kSB + (lane >> 4) * 4 + r;
                float v = acc[j][r] + bb;
                if (skip) v += skip[j][r];
                act[row * nn::kRS + co] = v > 0.0f ? v : 0.0f;
            }
}

__device__ __forceinline__ void read_skip(f32x4 (&skip)[nn::kTPW], const float* act, const int (&sq)[nn::kTPW], int lane,
                                          int nt, int ntiles) {
    const int co = nt * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < nn::kTPW; ++j)
        if (j < ntiles)
#pragma unroll
            for (int r = 0; r < 4; ++r) skip[j][r] = act[(sq[j] * nn::kSB + (lane >> 4) * 4 + r) * nn::kRS + co];
}

// value + policy heads (net.rs:152-213) for position `s` of the workgroup (one wave). ld(row, c)
// returns activation channel c of LDS row `row` (= square * 16 + position) as fp32.
template <class LD>
__device__ __forceinline__ void heads_g(const LD& ld, float* scratch, int s, const float* p, int lane, int b, int B,
                                        float* policy, float* value) {
    const float* vw = p;
    const float vb = p[64];
    const float* l1w = p + 68;
    const float* l1b = l1w + 64 * 25;
    const float* l2w = l1b + 64;
    const float l2b = l2w[64];
    const float* pp = p + nn::kValueF;
    const float pb0 = pp[128], pb1 = pp[129];
    const float* plw = pp + 132;
    const float* plb = plw + 2500;
    if (lane < 25) {  // 1x1 convs (value 64->1, policy 64->2) with folded BN, ReLU; lane = square
        float sv = vb, s0 = pb0, s1 = pb1;
        const int row = lane * nn::kSB + s;
        for (int c = 0; c < nn::kCh; c += 4) {
            float4 x;
            x.x = ld(row, c);
            x.y = ld(row, c + 1);
            x.z = ld(row, c + 2);
            x.w = ld(row, c + 3);
            sv += vw[c] * x.x + vw[c + 1] * x.y + vw[c + 2] * x.z + vw[c + 3] * x.w;
            s0 += pp[c] * x.x + pp[c + 1] * x.y + pp[c + 2] * x.z + pp[c + 3] * x.w;
            s1 += pp[64 + c] * x.x + pp[65 + c] * x.y + pp[66 + c] * x.z + pp[67 + c] * x.w;
        }
        scratch[lane] = sv > 0.0f ? sv : 0.0f;       // value features [25]
        scratch[32 + lane] = s0 > 0.0f ? s0 : 0.0f;  // policy features, flatten(1,-1) order
        scratch[57 + lane] = s1 > 0.0f ? s1 : 0.0f;
    }
    float hj = l1b[lane];
    for (int q = 0; q < 25; ++q) hj += l1w[q * 64 + lane] * scratch[q];  // l1w stored [25][64]
    hj = hj > 0.0f ? hj : 0.0f;
    const float vsum = wave_sum_f(l2w[lane] * hj);
    float lg = -INFINITY;
    if (lane < 50) {
        lg = plb[lane];
        for (int f = 0; f < 50; ++f) lg += plw[f * 50 + lane] * scratch[32 + f];  // plw stored [in][out]
    }
    const float mx = wave_max_f(lg);
    const float e = lane < 50 ? expf(lg - mx) : 0.0f;
    const float den = wave_sum_f(e);
    if (b < B) {
        if (lane < 50) policy[(size_t)b * 50 + lane] = e / den;
        if (lane == 0) value[b] = tanhf(vsum + l2b);
    }
}

// The heads after the 1x1 convs for NP positions of one wave: feat[q] = the q-th position's
// features, [0..24] value, [25..74] policy in flatten(1,-1) order (already bias + ReLU). Same
// arithmetic per position as heads_g's second half; the weights are read once for all NP
// positions and the NP dot products are independent chains.
template <int NP>
__device__ __forceinline__ void heads_mlp(const float* const (&feat)[NP], const int (&bs)[NP], const float* p, int lane,
                                          int B, float* policy, float* value) {
    const float* l1w = p + 68;
    const float* l1b = l1w + 64 * 25;
    const float* l2w = l1b + 64;
    const float l2b = l2w[64];
    const float* pp = p + nn::kValueF;
    const float* plw = pp + 132;
    const float* plb = plw + 2500;
    float hj[NP], lg[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) hj[q] = l1b[lane];
    for (int k = 0; k < 25; ++k) {
        const float w = l1w[k * 64 + lane];
#pragma unroll
        for (int q = 0; q < NP; ++q) hj[q] += w * feat[q][k];
    }
    const bool pl = lane < 50;
#pragma unroll
    for (int q = 0; q < NP; ++q) lg[q] = pl ? plb[lane] : -INFINITY;
    if (pl)
        for (int f = 0; f < 50; ++f) {
            const float w = plw[f * 50 + lane];
#pragma unroll
            for (int q = 0; q < NP; ++q) lg[q] += w * feat[q][25 + f];
        }
    const float w2 = l2w[lane];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const float h = hj[q] > 0.0f ? hj[q] : 0.0f;
        const float vsum = wave_sum_f(w2 * h);
        const float mx = wave_max_f(lg[q]);
        const float e = pl ? expf(lg[q] - mx) : 0.0f;
        const float den = wave_sum_f(e);
        if (bs[q] < B) {
            if (pl) policy[(size_t)bs[q] * 50 + lane] = e / den;
            if (lane == 0) value[bs[q]] = tanhf(vsum + l2b);
        }
    }
}

// Wave reductions on DPP within each 16-lane row (quad swaps, half-row and row mirrors) and four
// v_readlane for the rows: a few cycles per step instead of a ds_bpermute round trip per step.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);  // row_half_mirror
    v += dpp_mov<0x140>(v);  // row_mirror: every lane holds its row's sum
    return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    v = fmaxf(v, dpp_mov<0x4E>(v));
    v = fmaxf(v, dpp_mov<0x141>(v));
    v = fmaxf(v, dpp_mov<0x140>(v));
    return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}

// Heads MLPs as exact-fp32 MFMAs over the workgroup's 16 positions (8 waves): waves 0-3 the value
// hidden layer (K = 25 features, 16 units each), waves 4-7 the policy logits (K = 50, 16 logits
// each; logits 50..63 and K padding have zero weights). Each wave fetches only its B fragments
// (20 KB per workgroup instead of every wave reading all 16 KB of MLP weights). The results go to
// an LDS table [16][128] (64 hidden | 64 logits); then every wave finishes 2 positions with the
// lane = unit / logit: ReLU, the 64-term value dot + tanh, the 50-way softmax (DPP reductions).
struct HeadMM {
    float w[13];
    float b1, w2, bp, b2;
};
__device__ __forceinline__ void heads_mm_fetch(HeadMM& R, const float* p, int wave, int lane) {
    const float* l1w = p + 68;
    const float* l1b = l1w + 64 * 25;
    const float* l2w = l1b + 64;
    const float* plw = p + nn::kValueF + 132;
    const float* plb = plw + 2500;
    const int n = (wave & 3) * 16 + (lane & 15), kq = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 13; ++kk) {
        const int k = 4 * kk + kq;
        if (wave < 4)
            R.w[kk] = (kk < 7 && k < 25) ? l1w[k * 64 + n] : 0.0f;
        else
            R.w[kk] = (k < 50 && n < 50) ? plw[k * 50 + n] : 0.0f;
    }
    R.b1 = l1b[lane];
    R.w2 = l2w[lane];
    R.bp = plb[lane < 50 ? lane : 0];
    R.b2 = l2w[64];
}
__device__ __forceinline__ void heads_mm(const HeadMM& R, const float* feat, float* tab, int wave, int lane, int b0,
                                         int B, float* policy, float* value) {
    const int p = lane & 15, kq = lane >> 4;
    f32x4 acc = {};
    if (wave < 4) {
#pragma unroll
        for (int kk = 0; kk < 7; ++kk)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(feat[p * 80 + 4 * kk + kq], R.w[kk], acc, 0, 0, 0);
    } else {
#pragma unroll
        for (int kk = 0; kk < 13; ++kk) {
            const int f = 4 * kk + kq;
            const float a = f < 50 ? feat[p * 80 + 25 + f] : 0.0f;  // (the table's pad is not initialised)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, R.w[kk], acc, 0, 0, 0);
        }
    }
    // C/D: column = unit (lane & 15) of this wave's 16, rows = positions 4 * kq + r
#pragma unroll
    for (int r = 0; r < 4; ++r) tab[(4 * kq + r) * 128 + wave * 16 + p] = acc[r];
    __syncthreads();
    const bool pl = lane < 50;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int pos = wave + 8 * q;
        const float hj = tab[pos * 128 + lane] + R.b1;
        const float lg = pl ? tab[pos * 128 + 64 + lane] + R.bp : -INFINITY;
        const float h = hj > 0.0f ? hj : 0.0f;
        const float vsum = wave_sum_dpp(R.w2 * h);
        const float mx = wave_max_dpp(lg);
        const float e = pl ? expf(lg - mx) : 0.0f;
        const float den = wave_sum_dpp(e);
        const int b = b0 + pos;
        if (b < B) {
            if (pl) policy[(size_t)b * 50 + lane] = e / den;
            if (lane == 0) value[b] = tanhf(vsum + R.b2);
        }
    }
}

__device__ __forceinline__ void heads(const float* act, float* scratch, int s, const float* p, int lane, int b, int B,
                                      float* policy, float* value) {
    heads_g([&](int row, int c) { return act[row * nn::kRS + c]; }, scratch, s, p, lane, b, B, policy, value);
}

__global__ void __launch_bounds__(64 * nn::kWaves) k_nn_sq16(const oaz_state* __restrict__ states, int B,
                                                             const float* __restrict__ blob, int blocks,
                                                             float* __restrict__ policy,
                                                             float* __restrict__ value, TileMap tm) {
    constexpr int kImageFloats = nn::kSB * 25 * nn::kRS;
    __shared__ __attribute__((aligned(16))) float lds[nn::kLdsFloats];
    float* act = lds;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nt = wave & 3, grp = wave >> 2;
    const int ntiles = grp == 0 ? nn::kTPW : 25 - nn::kTPW;
    int sq[nn::kTPW];
#pragma unroll
    for (int j = 0; j < nn::kTPW; ++j) sq[j] = (j < ntiles) ? c_sq_order[grp * nn::kTPW + j] : 0;
    const TileSpan sp = tile_span(tm, B);
    const int b0 = sp.b0;
    B = sp.end;
    // per-position card/colour info for the first-layer table; the area is wave 0's head
    // scratch, free until the heads run
    int* pinfo = reinterpret_cast<int*>(lds + kImageFloats);

    // encoder (common.rs:26-80): lane = (position lane&15, bitboard lane>>4: red pawns, red
    // king, blue pawns, blue king); the cards / colour of each position go to LDS
    {
        const int pos = lane & 15, kq = lane >> 4;
        const int b = min(b0 + pos, sp.cap - 1);  // an empty tile of a bucket starts past cap
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&states[b]);
        const uint32_t bb = kq == 0 ? w[2] : kq == 1 ? w[0] : kq == 2 ? w[3] : w[1];
        if (tid < nn::kSB) {
            const oaz_state st = states[b];
            const int blue = st.to_move & 1;
            const int c0 = (blue ? st.cards[2] : st.cards[0]) & 15, c1 = (blue ? st.cards[3] : st.cards[1]) & 15;
            pinfo[tid] = c0 | (c1 << 4) | (blue << 8);
        }
        if (b0 >= B) return;  // an empty tile of a compacted bucket (uniform over the workgroup)
        __syncthreads();
        f32x4 acc[nn::kTPW];
#pragma unroll
        for (int j = 0; j < nn::kTPW; ++j) acc[j] = f32x4{};
        conv_l1(acc, bb, blob, sq, lane, nt, ntiles);
        conv_l1_const(acc, blob + nn::kL1B + nn::kCh, pinfo[lane & 15], sq, lane, nt, ntiles);
        epilogue(acc, act, blob + nn::kL1B, nullptr, sq, lane, nt, ntiles);
        __syncthreads();
    }

    const float* p = blob + nn::kL1B + nn::kCh + nn::kL1Table;
    f32x4 acc[nn::kTPW];
    f32x4 skip[nn::kTPW];
    auto conv = [&](const float* w) {
#pragma unroll
        for (int j = 0; j < nn::kTPW; ++j) acc[j] = f32x4{};
        conv64(acc, act, reinterpret_cast<const float4*>(w), sq, lane, nt, ntiles);
    };
    for (int blk = 0; blk < blocks; ++blk) {
        read_skip(skip, act, sq, lane, nt, ntiles);
        conv(p);  // small block 1: conv + BN + ReLU
        p += nn::kW64;
        __syncthreads();
        epilogue(acc, act, p, nullptr, sq, lane, nt, ntiles);
        p += nn::kCh;
        __syncthreads();
        conv(p);  // small block 2: conv + BN, + skip, ReLU
        p += nn::kW64;
        __syncthreads();
        epilogue(acc, act, p, skip, sq, lane, nt, ntiles);
        p += nn::kCh;
        __syncthreads();
    }
    float* scratch = lds + kImageFloats + wave * nn::kScratch;
    for (int s = wave; s < nn::kSB; s += nn::kWaves) heads(act, scratch, s, p, lane, b0 + s, B, policy, value);
}

// ---- fp32 split (OAZ_FP32_SPLIT): bf16x6 MFMA with fp32-level error ------------------------------
// Every fp32 operand x (activation or folded weight) is split EXACTLY into three bf16 terms,
// x = h + m + l: h = the top 16 bits of x (8 significant bits), m = the top 16 bits of x - h,
// l = x - h - m (both subtractions are exact and l has <= 8 significant bits). Of the nine
// products of a*b the six down to 2^-16 relative are computed (hh, hm, mh, hl, mm, lh) on
// v_mfma_f32_16x16x32_bf16, whose bf16 x bf16 products are exact in fp32 and which accumulates
// in fp32; the dropped ml + lm + ll are below 2^-23 relative, i.e. at fp32 rounding level
// (measured: errors vs a float64 forward equal the exact-fp32 kernel's).
// One K=32 block costs 6 x 16 cycles instead of 8 x 32 for v_mfma_f32_16x16x4_f32 (2.67x).
//
// Geometry = k_nn_sq16 (16 positions, square-major rows, 8 waves = 2 square groups x 4 N-tiles,
// off-board (square, tap) products skipped). The LDS image holds the three bf16 planes of every
// activation: row (square*16 + position) = [piece][64 channels] = 384 B, unpadded (153.6 KB);
// 16-byte chunk c (8 channels) of piece p of row r sits at chunk p*8 + (c ^ key(r)) (chunk_off):
// conflict-free A-fragment reads and epilogue stores.
namespace x6 {
// byte offset of an 8-channel chunk. Swizzle key ((row >> 1) ^ 4 (row & 1)) & 7: every 16-lane group of
// the A-fragment ds_read_b128s hits 16 distinct bank slots, and every 32-lane half of the
// epilogue's paired ds_write_b32s (rows 2k, 2k+1, 2k+4, 2k+5 x 16 channels) 32 distinct banks
// (with key (row >> 1) & 7 rows 2k and 2k+1 collided: a 2-way conflict on every store).
__device__ __forceinline__ int chunk_off(int row, int piece, int c8) {
    return row * kRowB + piece * 128 + ((c8 ^ (((row >> 1) ^ ((row & 1) << 2)) & 7)) << 4);
}
__device__ __forceinline__ void split3(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
    const uint32_t hb = __float_as_uint(v) & 0xffff0000u;
    const float r = v - __uint_as_float(hb);
    const uint32_t mb = __float_as_uint(r) & 0xffff0000u;
    const float lo = r - __uint_as_float(mb);
    h = (uint16_t)(hb >> 16);
    m = (uint16_t)(mb >> 16);
    l = (uint16_t)(__float_as_uint(lo) >> 16);
}
// byte offset of channel c of row r within its piece-0 plane; rows r and r + 16k share the
// swizzle, so the offset of (square sq, row-in-tile r) is sq * 16 * kRowB + elem_off(r, c)
__device__ __forceinline__ int elem_off(int row, int c) { return chunk_off(row, 0, c >> 3) + (c & 7) * 2; }
__device__ __forceinline__ void store_at(char* img, int o, float v) {
    uint16_t h, m, l;
    split3(v, h, m, l);
    *reinterpret_cast<uint16_t*>(img + o) = h;
    *reinterpret_cast<uint16_t*>(img + o + 128) = m;
    *reinterpret_cast<uint16_t*>(img + o + 256) = l;
}
__device__ __forceinline__ float load_at(const char* img, int o) {  // h + m + l = the fp32 value
    const float h = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(img + o) << 16);
    const float m = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(img + o + 128) << 16);
    const float l = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(img + o + 256) << 16);
    return h + (m + l);
}
__device__ __forceinline__ float load(const char* img, int row, int c) { return load_at(img, elem_off(row, c)); }
}  // namespace x6

// Square groups (compile-time) of the split kernels: the two waves of a SIMD (waves w and w + 4)
// own N-tile w & 3 of two disjoint square groups, cut unevenly from kSqOrderU (interior, corners,
// then edges): the older wave wins MFMA arbitration and runs ahead, the younger fills its gaps, so
// equal halves leave the younger finishing alone. GRP 3 / 4: 15 / 10 squares (109 / 60 on-board
// taps; k_nn_x6), GRP 7 / 8 and 9 / 10: k_nn_h3's (below).
constexpr int8_t kSqOrderU[25] = {6, 7, 8, 11, 12, 13, 16, 17, 18, 0, 4, 20, 24, 2, 22,
                                  1, 3, 5, 10, 9, 14, 15, 19, 21, 23};
// k_nn_h3's split: 17 / 8 in fp16x3 mode (GRP 7 / 8), 14 / 11 in bf16 mode (GRP 9 / 10). Same-box A/B
// (tools/ab_libs.sh; profiles/r03_nn_split_ab.log, r03_nn_h1split_ab.log): fp16x3 16 / 9 within noise
// of 17 / 8, 18 / 7 +1.2 %, 15 / 10 +0.2 %; bf16 6-block against 17 / 8: 16 / 9 -1.8 %, 15 / 10 -2.2 %,
// 14 / 11 -3.0 %, 13 / 12 -2.4 % (its single product leaves the partner wave less to fill).
#ifndef OAZ_H3_SPLIT
#define OAZ_H3_SPLIT 17
#endif
#ifndef OAZ_H3_KH
#define OAZ_H3_KH 4  // squares per batch (A fragments in flight per step run)
#endif
#ifndef OAZ_H1_PP
#define OAZ_H1_PP 1  // bf16 mode: two image buffers, the convs alternate (one barrier per conv)
#endif
#ifndef OAZ_H1_L1F16
#define OAZ_H1_L1F16 1  // bf16 mode: the first layer on fp16 MFMA (the fp16x3 mode's), not exact fp32 MFMA
#endif
#ifndef OAZ_H1_SPLIT
#define OAZ_H1_SPLIT 13
#endif
constexpr int kH3Split = OAZ_H3_SPLIT, kH1Split = OAZ_H1_SPLIT;
constexpr int grp_n(int grp) {
    return grp == 3 ? 15 : grp == 4 ? 10 : grp == 7 ? kH3Split : grp == 8 ? 25 - kH3Split : grp == 9 ? kH1Split
                                                                                                  : 25 - kH1Split;
}
constexpr int grp_first(int grp) { return grp == 4 ? 15 : grp == 8 ? kH3Split : grp == 10 ? kH1Split : 0; }
constexpr int grp_sq(int grp, int j) { return kSqOrderU[grp_first(grp) + j]; }

// On-board squares of group GRP for tap T: the conv is straight-line code per (group, tap), with no
// per-MFMA on-board tests.
struct TapList {
    int n;
    int8_t j[25];   // index into the group's square list (accumulator)
    int8_t nb[25];  // neighbour square read for that tap
};
constexpr TapList tap_list(int grp, int t) {
    TapList L{};
    for (int j = 0; j < grp_n(grp); ++j) {
        const int sq = grp_sq(grp, j);
        const int r = sq / 5 + t / 3 - 1, c = sq % 5 + t % 3 - 1;
        if (r >= 0 && r < 5 && c >= 0 && c < 5) {
            L.j[L.n] = (int8_t)j;
            L.nb[L.n] = (int8_t)(r * 5 + c);
            ++L.n;
        }
    }
    return L;
}

// Batch plan: the 18 (tap, K-half) steps cut into near-equal batches of <= KH on-board squares.
struct X6Batch {
    int t, m, n;
    int8_t j[16], nb[16];
};
struct X6Plan {
    int nbat;
    X6Batch b[96];
};
constexpr X6Plan x6_plan(int grp, int kh) {
    X6Plan P{};
    for (int s = 0; s < 18; ++s) {
        const TapList L = tap_list(grp, s / 2);
        const int nb = (L.n + kh - 1) / kh;
        int q = 0;
        for (int k = 0; k < nb; ++k) {
            const int n = (L.n - q) / (nb - k);  // near-equal split, larger batches last
            X6Batch B{};
            B.t = s / 2;
            B.m = s % 2;
            B.n = n;
            for (int i = 0; i < n; ++i) {
                B.j[i] = L.j[q + i];
                B.nb[i] = L.nb[q + i];
            }
            q += n;
            P.b[P.nbat++] = B;
        }
    }
    return P;
}
template <int GRP, int KH>
struct X6PlanOf {
    static constexpr X6Plan P = x6_plan(GRP, KH);
};

// k_nn_h3 plan: the 18 (tap, K-half) steps of the group cut into batches of <= KH squares. first:
// the batch starts a step run (its B pieces were prefetched); nstep: the step of the next run (its B
// pieces are prefetched now).
struct H3Batch {
    int t, m, n, first, nstep;
    int8_t j[16], nb[16];
};
struct H3Plan {
    int nbat;
    H3Batch b[96];
};
constexpr H3Plan h3_plan(int grp, int kh) {
    H3Plan P{};
    for (int s = 0; s < 18; ++s) {  // step = tap * 2 + K-half
        const TapList L = tap_list(grp, s / 2);
        const int nb = (L.n + kh - 1) / kh;
        int q = 0;
        for (int k = 0; k < nb; ++k) {
            const int m = (L.n - q) / (nb - k);  // near-equal split, larger batches last
            H3Batch B{};
            B.t = s / 2;
            B.m = s % 2;
            B.n = m;
            B.first = k == 0;
            B.nstep = -1;
            for (int i = 0; i < m; ++i) {
                B.j[i] = L.j[q + i];
                B.nb[i] = L.nb[q + i];
            }
            q += m;
            P.b[P.nbat++] = B;
        }
    }
    int next = -1;
    for (int k = P.nbat - 1; k >= 0; --k)
        if (P.b[k].first) {
            P.b[k].nstep = next;
            next = P.b[k].t * 2 + P.b[k].m;
        }
    return P;
}
template <int GRP, int KH>
struct H3PlanOf {
    static constexpr H3Plan P = h3_plan(GRP, KH);
};

// Kernel configurations (8 waves: two per SIMD, square groups GRP0 / GRP1 x 4 N-tiles, <= 256 VGPRs;
// KH: squares per batch of A fragments). DBG (diagnostic builds only, `make AB=1`; timing only, wrong
// results): 2 per-wave s_memtime phase sums written over the first policy rows (tools/nn_phases.py),
// 3 no conv A reads, 4 no conv B loads, 7 conv B loads of one step, 9 conv A reads discarded (ablations),
// 5 workgroup start / end stamps
// (tools/nn_timeline.py).
template <int DBG_ = 0>
struct X6Cfg {  // k_nn_x6 (OAZ_FP32_SPLIT, and k_nn_h3's fp16-range recompute): 15 / 10 squares
    static constexpr int WAVES = 8, KH = OAZ_H3_KH, NS = 15, GRP0 = 3, GRP1 = 4, TR = 0, DBG = DBG_;
};
template <int BF_, int DBG_ = 0>
struct H3Cfg {  // k_nn_h3: 17 / 8 squares (bf16: 13 / 12); BF: OAZ_BF16 mode (one bf16 piece, one product; C5)
    static constexpr int kSplit = BF_ ? kH1Split : kH3Split;
    static constexpr int WAVES = 8, KH = OAZ_H3_KH, NS = kSplit > 12 ? kSplit : 25 - kSplit, GRP0 = BF_ ? 9 : 7,
                         GRP1 = BF_ ? 10 : 8, TR = 1, BF = BF_, DBG = DBG_;
};

// A-fragment loads / MFMAs of batch K (compile-time: the LDS address is one of six per-lane bases
// ab[m][seg] = lo[m] + seg * 64 KiB plus an immediate offset < 64 KiB)
template <int GRP, int KH, int K, int N>
__device__ __forceinline__ void x6_load(bf16x8 (&a)[N], const char* img, const int (&ab)[2][3], int piece) {
    constexpr X6Batch B = X6PlanOf<GRP, KH>::P.b[K];
#pragma unroll
    for (int q = 0; q < N; ++q)
        if (q < B.n) {
            const int off = B.nb[q] * (nn::kSB * x6::kRowB) + piece * 128;  // folds to a constant
            a[q] = *reinterpret_cast<const bf16x8*>(img + ab[B.m][off >> 16] + (off & 0xffff));
        }
}

template <int GRP, int KH, int K, int NS, int N>
__device__ __forceinline__ void x6_mfma(f32x4 (&acc)[NS], const bf16x8 (&a)[N], const bf16x8& bv) {
    constexpr X6Batch B = X6PlanOf<GRP, KH>::P.b[K];
#pragma unroll
    for (int q = 0; q < N; ++q)
        if (q < B.n) acc[B.j[q]] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[q], bv, acc[B.j[q]], 0, 0, 0);
}

// B pieces of (tap, K-half) step S for N-tile nt: [step][piece][N-tile][lane] bf16x8, read with
// buffer loads (descriptor + one per-lane VGPR offset + a constant SGPR offset: no 64-bit vector
// address arithmetic per load)
struct X6W {
    __amdgpu_buffer_rsrc_t r;
    int voff;  // (nt * 64 + lane) * 16
};
__device__ __forceinline__ X6W x6_w(const float* p, int lane, int nt) {
    X6W w;
    w.r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(x6::kW * 4), 0x00020000);
    w.voff = (nt * 64 + lane) * 16;
    return w;
}
__device__ __forceinline__ bf16x8 x6_ldb(const X6W& w, int entry) {  // entry = (step * 3 + piece) * 4
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w.r, w.voff, entry * 64 * 16, 0));
}

template <class C, int GRP, int K>
__device__ __forceinline__ void x6_step_b(const X6W& W, bf16x8 (&b)[3], bf16x8 (&bn)[3]) {
    constexpr const X6Plan& P = X6PlanOf<GRP, C::KH>::P;
    constexpr X6Batch B = P.b[K];
    constexpr int step = B.t * 2 + B.m;
    constexpr bool first_of_step = K == 0 || P.b[K - 1].t * 2 + P.b[K - 1].m != step;
    if constexpr (first_of_step && K > 0) {
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) b[pc] = bn[pc];
    }
    if constexpr (first_of_step && step + 1 < 18) {  // prefetch the next step's B pieces
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) bn[pc] = x6_ldb(W, ((step + 1) * 3 + pc) * 4);
    }
}

// PIPE 1, batch K (X holds its m pieces on entry and the next batch's on exit; X/Y swap roles
// with K's parity):
//   load Y = h | m*Bh, m*Bm | load X = l | h*Bh, h*Bm, h*Bl | load Y = next m | l*Bh
template <class C, int GRP, int K>
__device__ __forceinline__ void conv_x6_batch(f32x4 (&acc)[C::NS], const char* img, const X6W& W,
                                              bf16x8 (&b)[3], bf16x8 (&bn)[3], bf16x8 (&X)[C::KH],
                                              bf16x8 (&Y)[C::KH], const int (&ab)[2][3]) {
    constexpr int KH = C::KH, NS = C::NS;
    x6_step_b<C, GRP, K>(W, b, bn);
    x6_load<GRP, KH, K>(Y, img, ab, 0);
    x6_mfma<GRP, KH, K, NS>(acc, X, b[0]);  // mh
    x6_mfma<GRP, KH, K, NS>(acc, X, b[1]);  // mm
    x6_load<GRP, KH, K>(X, img, ab, 2);
    x6_mfma<GRP, KH, K, NS>(acc, Y, b[0]);  // hh
    x6_mfma<GRP, KH, K, NS>(acc, Y, b[1]);  // hm
    x6_mfma<GRP, KH, K, NS>(acc, Y, b[2]);  // hl
    if constexpr (K + 1 < X6PlanOf<GRP, KH>::P.nbat) x6_load<GRP, KH, K + 1>(Y, img, ab, 1);
    x6_mfma<GRP, KH, K, NS>(acc, X, b[0]);  // lh
    __builtin_amdgcn_sched_barrier(0);      // bound the live ranges: no loads hoisted across batches
}

template <class C, int GRP, int... K>
__device__ __forceinline__ void conv_x6_run(f32x4 (&acc)[C::NS], const char* img, const X6W& W, const int (&lo)[2],
                                            std::integer_sequence<int, K...>) {
    int ab[2][3];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int sg = 0; sg < 3; ++sg) ab[m][sg] = lo[m] + sg * 65536;
    bf16x8 b[3], bn[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) b[pc] = x6_ldb(W, pc * 4);
    bf16x8 X[C::KH], Y[C::KH];
    x6_load<GRP, C::KH, 0>(X, img, ab, 1);
    ((K % 2 == 0 ? conv_x6_batch<C, GRP, K>(acc, img, W, b, bn, X, Y, ab)
                 : conv_x6_batch<C, GRP, K>(acc, img, W, b, bn, Y, X, ab)),
     ...);
}

// bias (+ residual), ReLU, split into the three LDS planes; C/D layout as in epilogue<>. Lanes co
// (even) and co^1 hold the same rows: the even lane stores rows 0 and 2, the odd lane rows 1 and
// 3, each as (even channel, odd channel) bf16 pairs per piece; eo[k] = elem_off(row of store k,
// co & ~1). ADD: add the residual held in `skip`; KEEP: the result is the next block's input, keep
// it in `skip` (every conv maps (square, position, channel) to the same lane and register, so the
// residual is never read back from the split LDS image).
template <class C, int GRP>
__device__ __forceinline__ void epilogue_x6_pack(const f32x4 (&acc)[C::NS], uint32_t (&pk)[C::NS][2][3],
                                                 const float* bias, f32x4 (&skip)[C::NS], int co, bool add,
                                                 bool keep) {
    const float bb = bias[co];
    const bool odd = co & 1;
    const float addf = add ? 1.0f : 0.0f;  // fma(skip, addf, v) = v + skip or v, exactly
    const uint32_t sel = odd ? 0x03020706u : 0x07060302u;
#pragma unroll
    for (int j = 0; j < grp_n(GRP); ++j) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = __builtin_fmaf(skip[j][r], addf, acc[j][r] + bb);
            v[r] = v[r] > 0.0f ? v[r] : 0.0f;
            if (keep) skip[j][r] = v[r];
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            // 2x2 transpose of (rows 2k, 2k+1) x (channels co&~1, co|1) between the lane pair:
            // one DPP swap (quad_perm [1,0,3,2]); then per piece one v_perm_b32 packs the two
            // bf16 (high halves) in channel order, its selector depending on the lane's parity
            const float keep_ = odd ? v[2 * k + 1] : v[2 * k];  // stays in this lane
            const float send = odd ? v[2 * k] : v[2 * k + 1];   // goes to the partner
            const float got = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(send), 0xB1, 0xF, 0xF, false));
            const uint32_t ka = __float_as_uint(keep_), ga = __float_as_uint(got);
            const float kr = keep_ - __uint_as_float(ka & 0xffff0000u), gr = got - __uint_as_float(ga & 0xffff0000u);
            const uint32_t kb = __float_as_uint(kr), gb = __float_as_uint(gr);
            const float kl = kr - __uint_as_float(kb & 0xffff0000u), gl = gr - __uint_as_float(gb & 0xffff0000u);
            pk[j][k][0] = __builtin_amdgcn_perm(ga, ka, sel);
            pk[j][k][1] = __builtin_amdgcn_perm(gb, kb, sel);
            pk[j][k][2] = __builtin_amdgcn_perm(__float_as_uint(gl), __float_as_uint(kl), sel);
        }
    }
}
template <class C, int GRP>
__device__ __forceinline__ void epilogue_x6_store(const uint32_t (&pk)[C::NS][2][3], char* img, const int (&eo)[2]) {
#pragma unroll
    for (int j = 0; j < grp_n(GRP); ++j)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            uint32_t* d = reinterpret_cast<uint32_t*>(img + grp_sq(GRP, j) * (nn::kSB * x6::kRowB) + eo[k]);
            d[0] = pk[j][k][0];
            d[32] = pk[j][k][1];
            d[64] = pk[j][k][2];
        }
}
// bias (+ residual), ReLU, split into the three LDS planes; C/D layout as in epilogue<>. Lanes co
// (even) and co^1 hold the same rows: the even lane stores rows 0 and 2, the odd lane rows 1 and
// 3, each as (even channel, odd channel) bf16 pairs per piece; eo[k] = elem_off(row of store k,
// co & ~1). ADD: add the residual held in `skip`; KEEP: the result is the next block's input, keep
// it in `skip` (every conv maps (square, position, channel) to the same lane and register, so the
// residual is never read back from the split LDS image). The VALU part (_pack) runs before the
// barrier that ends the conv's reads, so a wave that finishes its MFMAs early packs while its SIMD
// partner still computes; only the stores (_store) wait for the barrier.
template <class C, int GRP>
__device__ __forceinline__ void epilogue_x6(const f32x4 (&acc)[C::NS], char* img, const float* bias,
                                            f32x4 (&skip)[C::NS], const int (&eo)[2], int co, bool add, bool keep) {
    uint32_t pk[C::NS][2][3];
    epilogue_x6_pack<C, GRP>(acc, pk, bias, skip, co, add, keep);
    epilogue_x6_store<C, GRP>(pk, img, eo);
}

// First layer (exact fp32 MFMA on 0/1 inputs, as k_nn_sq16): 4 bitboards x on-board taps, then the
// constant planes (the mover's two cards, blue-to-move) as 5 k-steps against the per-square table.
// Its weights do not depend on the positions, so they are requested (first_layer_x6_fetch) before
// the positions are read, and their latency overlaps the state load.
template <int GRP>
struct L1Regs {
    float w[9];  // bitboard weights per tap (lane: plane kq, channel co)
};
template <int GRP>
__device__ __forceinline__ void first_layer_x6_fetch(L1Regs<GRP>& R, const float* W, int lane, int nt) {
#pragma unroll
    for (int t = 0; t < 9; ++t) R.w[t] = W[(t * 4 + nt) * 64 + lane];
}
template <class C, int GRP>
__device__ __forceinline__ void first_layer_x6(f32x4 (&acc)[C::NS], const L1Regs<GRP>& R, const float* table,
                                               uint32_t bb, int cinfo, int lane, int nt) {
    const int kq = lane >> 4, co = nt * 16 + (lane & 15);
    constexpr int kBatch = 5;  // squares whose table rows are requested together
    float tb[kBatch][5];
    auto fetch = [&](int j0) {
#pragma unroll
        for (int q = 0; q < kBatch; ++q)
            if (j0 + q < grp_n(GRP)) {
                const float* ts = table + (size_t)grp_sq(GRP, j0 + q) * 17 * nn::kCh + co;
#pragma unroll
                for (int st = 0; st < 5; ++st) {
                    const int k = 4 * st + kq;
                    tb[q][st] = k < 17 ? ts[k * nn::kCh] : 0.0f;
                }
            }
    };
    fetch(0);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < grp_n(GRP); ++j) {
            const int sq = grp_sq(GRP, j);
            const int r = sq / 5 + t / 3 - 1, c = sq % 5 + t % 3 - 1;
            if (r >= 0 && r < 5 && c >= 0 && c < 5) {
                const float a = (float)((bb >> (31 - (r * 5 + c))) & 1u);
                acc[j] = C::TR ? __builtin_amdgcn_mfma_f32_16x16x4f32(R.w[t], a, acc[j], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_16x16x4f32(a, R.w[t], acc[j], 0, 0, 0);
            }
        }
    const int c0 = cinfo & 15, c1 = (cinfo >> 4) & 15, blue = (cinfo >> 8) & 1;
    float a[5];
#pragma unroll
    for (int st = 0; st < 5; ++st) {
        const int k = 4 * st + kq;
        a[st] = k < 16 ? ((k == c0 || k == c1) ? 1.0f : 0.0f) : (k == 16 ? (float)blue : 0.0f);
    }
#pragma unroll
    for (int j0 = 0; j0 < grp_n(GRP); j0 += kBatch) {
#pragma unroll
        for (int st = 0; st < 5; ++st)
#pragma unroll
            for (int q = 0; q < kBatch; ++q)
                if (j0 + q < grp_n(GRP))
                    acc[j0 + q] = C::TR
                                      ? __builtin_amdgcn_mfma_f32_16x16x4f32(tb[q][st], a[st], acc[j0 + q], 0, 0, 0)
                                      : __builtin_amdgcn_mfma_f32_16x16x4f32(a[st], tb[q][st], acc[j0 + q], 0, 0, 0);
        if (j0 + kBatch < grp_n(GRP)) fetch(j0 + kBatch);
    }
}

// The whole forward for the waves of square group GRP.
template <class C, int GRP>
__device__ __forceinline__ void nn_x6_body(const oaz_state* __restrict__ states, const TileSpan sp,
                                           const float* __restrict__ blob, int blocks, float* __restrict__ policy,
                                           float* __restrict__ value, float* lds) {
    const int B = sp.end;
    constexpr int NS = C::NS;
    char* img = reinterpret_cast<char*>(lds);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nt = wave & 3;
    const int b0 = sp.b0;
    int* pinfo = reinterpret_cast<int*>(lds + x6::kImageB / 4);
    const int co = nt * 16 + (lane & 15);
    const int i = lane & 15, kq = lane >> 4;
    int eo[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) eo[k] = x6::elem_off(kq * 4 + 2 * k + (co & 1), co & ~1);
    const int lo[2] = {x6::chunk_off(i, 0, kq), x6::chunk_off(i, 0, 4 + kq)};

    f32x4 acc[NS];
    f32x4 skip[NS];
    uint64_t ph[6] = {0, 0, 0, 0, 0, 0};  // DBG 2: first layer, conv, barrier 1, epilogue, barrier 2, heads
    uint64_t tm = C::DBG == 2 ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) {
        if constexpr (C::DBG == 2) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph[k] += t - tm;
            tm = t;
        }
    };
    {  // encoder + first layer
        L1Regs<GRP> l1;
        first_layer_x6_fetch<GRP>(l1, blob, lane, nt);
        const int b = min(b0 + i, sp.cap - 1);  // an empty tile of a bucket starts past cap
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&states[b]);
        const uint32_t bb = kq == 0 ? w[2] : kq == 1 ? w[0] : kq == 2 ? w[3] : w[1];
        if (tid < nn::kSB) {
            const oaz_state st = states[b];
            const int blue = st.to_move & 1;
            const int c0 = (blue ? st.cards[2] : st.cards[0]) & 15, c1 = (blue ? st.cards[3] : st.cards[1]) & 15;
            pinfo[tid] = c0 | (c1 << 4) | (blue << 8);
        }
        if (b0 >= B) return;  // an empty tile of a compacted bucket (uniform over the workgroup)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NS; ++j) acc[j] = skip[j] = f32x4{};  // skip: finite for the fma in epilogue_x6
        first_layer_x6<C, GRP>(acc, l1, blob + nn::kL1B + nn::kCh, bb, pinfo[i], lane, nt);
        epilogue_x6<C, GRP>(acc, img, blob + nn::kL1B, skip, eo, co, false, true);
        __syncthreads();
    }
    // 2 * blocks convs through one call site (small block 1: conv + BN + ReLU; small block 2:
    // conv + BN, + skip, ReLU)
    stamp(0);
    const float* p = blob + nn::kL1B + nn::kCh + nn::kL1Table;
    for (int c = 0; c < 2 * blocks; ++c) {
#pragma unroll
        for (int j = 0; j < NS; ++j) acc[j] = f32x4{};
        conv_x6_run<C, GRP>(acc, img, x6_w(p, lane, nt), lo,
                            std::make_integer_sequence<int, X6PlanOf<GRP, C::KH>::P.nbat>{});
        stamp(1);
        p += x6::kW;
        uint32_t pk[NS][2][3];
        epilogue_x6_pack<C, GRP>(acc, pk, p, skip, co, c & 1, c & 1);
        stamp(3);
        __syncthreads();
        stamp(2);
        epilogue_x6_store<C, GRP>(pk, img, eo);
        stamp(3);
        p += nn::kCh;
        __syncthreads();
        stamp(4);
    }
    // heads: the value / policy 1x1 convs as split-fp32 MFMAs on the LDS image (one 16x16 tile
    // per square: rows = positions, columns 0 / 1 / 2 = value, policy planes 0 / 1), then the MLPs
    // per position on the VALU from a feature table in LDS
    {
        const bf16x8* HB = reinterpret_cast<const bf16x8*>(p + nn::kValueF + nn::kPolicyF);
        bf16x8 hb[2][3];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) hb[m][pc] = HB[(m * 3 + pc) * 64 + lane];
        constexpr int kSqPerWave = (25 + C::WAVES - 1) / C::WAVES;
        f32x4 hacc[kSqPerWave];
#pragma unroll
        for (int q = 0; q < kSqPerWave; ++q) {
            hacc[q] = f32x4{};
            const int sq = wave + q * C::WAVES;
            if (sq < 25) {
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const char* a = img + sq * (nn::kSB * x6::kRowB) + lo[m];
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(a);
                    const bf16x8 am = *reinterpret_cast<const bf16x8*>(a + 128);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(a + 256);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, hb[m][0], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, hb[m][1], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[m][0], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[m][1], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[m][2], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, hb[m][0], hacc[q], 0, 0, 0);
                }
            }
        }
        __syncthreads();  // the image is no longer read: its first 4.8 KB become the feature table
        float* feat = reinterpret_cast<float*>(img);  // [16 positions][80]
        const float hbias = i == 0 ? p[64] : i == 1 ? p[nn::kValueF + 128] : p[nn::kValueF + 129];
#pragma unroll
        for (int q = 0; q < kSqPerWave; ++q) {
            const int sq = wave + q * C::WAVES;
            if (sq < 25 && i < 3)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = hacc[q][r] + hbias;
                    feat[(kq * 4 + r) * 80 + i * 25 + sq] = v > 0.0f ? v : 0.0f;
                }
        }
        __syncthreads();
        constexpr int NP = nn::kSB / C::WAVES;  // positions per wave
        const float* fq[NP];
        int bq[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            fq[q] = feat + (wave + q * C::WAVES) * 80;
            bq[q] = b0 + wave + q * C::WAVES;
        }
        heads_mlp<NP>(fq, bq, p, lane, B, policy, value);
    }
    if constexpr (C::DBG == 2) {
        stamp(5);
        __syncthreads();
        if (lane < 6 && b0 + nn::kSB <= B) policy[(size_t)b0 * 50 + wave * 6 + lane] = (float)ph[lane];
    }
}

template <class C>
__global__ void __launch_bounds__(64 * C::WAVES) k_nn_x6(const oaz_state* __restrict__ states, int B,
                                                        const float* __restrict__ blob, int blocks,
                                                        float* __restrict__ policy, float* __restrict__ value,
                                                        TileMap tm) {
    __shared__ __attribute__((aligned(16))) float lds[x6::kLdsFloats];
    const TileSpan sp = tile_span(tm, B);
    if ((threadIdx.x >> 8) == 0) {  // waves 0-3: the bigger square group, ahead in MFMA arbitration
        __builtin_amdgcn_s_setprio(1);
        nn_x6_body<C, C::GRP0>(states, sp, blob, blocks, policy, value, lds);
    } else {
        nn_x6_body<C, C::GRP1>(states, sp, blob, blocks, policy, value, lds);
    }
}

// ---- fp32 split over fp16 (OAZ_FP32_SPLIT16): three f16 MFMA products per fp32 MAC -----------------
// Every fp32 operand x is split into two fp16 terms, hi = fp16(x) (round to nearest even) and
// lo = fp16(x - hi) (x - hi is exact in fp32): hi + lo carries 22 significant bits. Of the four
// products the three down to 2^-22 relative are computed (hi*hi, hi*lo, lo*hi) on
// v_mfma_f32_16x16x32_f16 (fp16 x fp16 products are exact in fp32, fp32 accumulation); lo*lo is
// below 2^-22 relative. One K=32 block costs 3 x 16 cycles (half of k_nn_x6's six products).
// fp16's exponent range is the price: conv weights are scaled per output channel by a power of two
// s (max |w s| in [2^14, 2^15), exact) and the epilogue multiplies by 1/s (exact); activations below 2^-14
// fall into fp16 subnormals (absolute error <= 2^-25 per term, below the fp32 rounding of the dot
// products); an activation >= 65504 would overflow, so every lane tracks the largest value it
// splits and raises range_flag (the engine reports OAZ_ERR_RANGE, never a silent result).
// Geometry, batch plans and pipelining as k_nn_x6. The LDS image holds two piece planes
// [piece][row][64 channels] (row = square*16 + position, 128 B); the 16-byte chunk c of row r sits
// at c ^ key(r), an XOR-linear key on the row bits found by exhaustive search
// (tools/h3_swizzle.py): conflict-free A-fragment ds_read_b128s and epilogue ds_write_b32s.
// PF: the B pieces of each conv's first step run are requested during the previous phase's
// epilogue (h3_first_b); same-box A/B -0.6 % (fp16x3) / -1.4 % (bf16 6-block) per launch. The
// phase-stamp build (DBG 2) keeps the old order: with both, its stamps make the allocator spill.
#ifndef OAZ_H3_PF
#define OAZ_H3_PF 1
#endif
template <class C>
constexpr bool h3_pf() { return OAZ_H3_PF && C::DBG != 2; }
namespace h3 {
__device__ __forceinline__ int key(int r) {
    return ((r & 1) << 1) ^ ((r >> 1) & 1) ^ (((r >> 2) & 1) << 2) ^ (((r >> 3) & 1) << 1);
}
__device__ __forceinline__ int chunk_off(int row, int c8) { return row * kRowB + ((c8 ^ key(row)) << 4); }
__device__ __forceinline__ int elem_off(int row, int c) { return chunk_off(row, c >> 3) + (c & 7) * 2; }
}  // namespace h3

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <class C, int GRP>
using H3P = H3PlanOf<GRP, C::KH>;

// A-fragment loads / MFMAs of batch K; the LDS address is one of four per-lane bases
// ab[m][seg] = lo[m] + seg * 64 KiB plus an immediate offset < 64 KiB (piece 1 = + kPlaneB)
template <class C, int GRP, int K, int N>
__device__ __forceinline__ void h3_load(f16x8 (&a)[N], const char* img, const int (&ab)[2][2], int piece) {
    if constexpr (C::DBG == 3 && K > 1) return;  // ablation (timing only, wrong results): no A reads
    constexpr H3Batch B = H3P<C, GRP>::P.b[K];
#pragma unroll
    for (int q = 0; q < N; ++q)
        if (q < B.n) {
            const int off = B.nb[q] * (nn::kSB * h3::kRowB) + piece * h3::kPlaneB;  // folds to a constant
            const f16x8 v = *reinterpret_cast<const f16x8*>(img + ab[B.m][off >> 16] + (off & 0xffff));
            if constexpr (C::DBG == 9 && K > 1)  // ablation: the A reads happen, the MFMAs keep stale operands
                asm volatile("" ::"v"(v));
            else
                a[q] = v;
        }
}

// Transposed C/D tiles: the operands swapped (weights as A, positions as B), so a lane holds the
// position lane & 15 and the channels 4 * (lane >> 4) + r of the N-tile -- the A/B fragment layouts
// of 16x16x32 are symmetric, so the same registers serve either order.
template <class C, int GRP, int K, int N>
__device__ __forceinline__ void h3_mfma(f32x4 (&acc)[C::NS], const f16x8 (&a)[N], const f16x8& bv) {
    constexpr H3Batch B = H3P<C, GRP>::P.b[K];
#pragma unroll
    for (int q = 0; q < N; ++q)
        if (q < B.n)
            acc[B.j[q]] = C::BF ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bv),
                                                                          __builtin_bit_cast(bf16x8, a[q]), acc[B.j[q]],
                                                                          0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x32_f16(bv, a[q], acc[B.j[q]], 0, 0, 0);
}

// B pieces of (tap, K-half) step S for N-tile nt: [step][piece][N-tile][lane] f16x8, buffer loads
__device__ __forceinline__ X6W h3_w(const float* p, int lane, int nt, int bytes = (int)(h3::kW * 4)) {
    X6W w;
    w.r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
    w.voff = (nt * 64 + lane) * 16;
    return w;
}
__device__ __forceinline__ f16x8 h3_ldb(const X6W& w, int entry) {  // entry = (step * 2 + piece) * 4
    return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(w.r, w.voff, entry * 64 * 16, 0));
}

// B pieces: b = the current step run's, bn = the next run's (loaded one step run ahead)
template <class C, int GRP, int K>
__device__ __forceinline__ void h3_step_b(const X6W& W, f16x8 (&b)[2], f16x8 (&bn)[2]) {
    constexpr H3Batch B = H3P<C, GRP>::P.b[K];
    if constexpr (B.first && K > 0) {
        b[0] = bn[0];
        b[1] = bn[1];
    }
    if constexpr (B.first && B.nstep >= 0 && C::DBG != 4) {  // prefetch the next step run's B pieces
                                                              // (DBG 4: ablation, no B loads)
        constexpr int ns = C::DBG == 7 ? 0 : B.nstep;  // ablation 7: every step reads step 0's pieces (L1 hits)
        if constexpr (C::BF) {  // BF: [step][N-tile][lane] bf16x8, one piece
            bn[0] = h3_ldb(W, ns * 4);
        } else {
            bn[0] = h3_ldb(W, (ns * 2 + 0) * 4);
            bn[1] = h3_ldb(W, (ns * 2 + 1) * 4);
        }
    }
}

// BF batch K: one piece, one product; the next batch's fragments load during this one's MFMAs
// (two buffers, roles swap with K's parity)
template <class C, int GRP, int K>
__device__ __forceinline__ void conv_h1_batch(f32x4 (&acc)[C::NS], const char* img, const X6W& W, f16x8 (&b)[2],
                                              f16x8 (&bn)[2], f16x8 (&X)[C::KH], f16x8 (&Xn)[C::KH],
                                              const int (&ab)[2][2]) {
    h3_step_b<C, GRP, K>(W, b, bn);
    if constexpr (K + 1 < H3P<C, GRP>::P.nbat) h3_load<C, GRP, K + 1>(Xn, img, ab, 0);
    h3_mfma<C, GRP, K>(acc, X, b[0]);
    __builtin_amdgcn_sched_barrier(0);
}

// fp16x3 batch K (X holds its lo pieces on entry and the next batch's on exit):
//   load Y = hi | lo*Bhi | load X = next lo | hi*Bhi, hi*Blo
template <class C, int GRP, int K>
__device__ __forceinline__ void conv_h3_batch(f32x4 (&acc)[C::NS], const char* img, const X6W& W, f16x8 (&b)[2],
                                              f16x8 (&bn)[2], f16x8 (&X)[C::KH], f16x8 (&Y)[C::KH],
                                              const int (&ab)[2][2]) {
    h3_step_b<C, GRP, K>(W, b, bn);
    h3_load<C, GRP, K>(Y, img, ab, 0);
    h3_mfma<C, GRP, K>(acc, X, b[0]);  // lo*hi
    if constexpr (K + 1 < H3P<C, GRP>::P.nbat) h3_load<C, GRP, K + 1>(X, img, ab, 1);
    h3_mfma<C, GRP, K>(acc, Y, b[0]);  // hi*hi
    h3_mfma<C, GRP, K>(acc, Y, b[1]);  // hi*lo
    __builtin_amdgcn_sched_barrier(0);  // bound the live ranges: no loads hoisted across batches
}

// The B pieces of a conv's first step run, requested before the previous phase's epilogue and
// barriers (their L2 latency would otherwise stall both waves of the SIMD at every conv's start).
template <class C, int GRP>
__device__ __forceinline__ void h3_first_b(f16x8 (&b)[2], const X6W& W) {
    constexpr H3Batch B0 = H3P<C, GRP>::P.b[0];
    if constexpr (C::BF) {
        b[0] = h3_ldb(W, (B0.t * 2 + B0.m) * 4);
        b[1] = b[0];
    } else {
        b[0] = h3_ldb(W, ((B0.t * 2 + B0.m) * 2 + 0) * 4);
        b[1] = h3_ldb(W, ((B0.t * 2 + B0.m) * 2 + 1) * 4);
    }
}

template <class C, int GRP, int... K>
__device__ __forceinline__ void conv_h3_run(f32x4 (&acc)[C::NS], const char* img, const X6W& W, const int (&lo)[2],
                                            const f16x8 (&bfirst)[2], std::integer_sequence<int, K...>) {
    int ab[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) ab[m][sg] = lo[m] + sg * 65536;
    f16x8 b[2] = {bfirst[0], bfirst[1]}, bn[2];
    if constexpr (!h3_pf<C>()) h3_first_b<C, GRP>(b, W);
    if constexpr (C::BF) {
        f16x8 X[C::KH], X2[C::KH];
        h3_load<C, GRP, 0>(X, img, ab, 0);
        ((K % 2 == 0 ? conv_h1_batch<C, GRP, K>(acc, img, W, b, bn, X, X2, ab)
                     : conv_h1_batch<C, GRP, K>(acc, img, W, b, bn, X2, X, ab)),
         ...);
    } else {
        f16x8 X[C::KH], Y[C::KH];
        h3_load<C, GRP, 0>(X, img, ab, 1);
        (conv_h3_batch<C, GRP, K>(acc, img, W, b, bn, X, Y, ab), ...);
    }
}

// Epilogue: the lane holds 4 consecutive channels (4 * kq + r of the N-tile) of one position,
// so no lane exchange is needed: bias / scale per register, the pair splits are packed
// conversions (v_cvt_pk_f16_f32, RNE), lo = fp16(fma(hi, -1, v)) (x - hi is exact in fp32, one
// rounding: v_fma_mix), and each piece is one 8-byte store per square.
// lo = fp16(v - hi) for a pair: v_fma_mix{lo,hi}_f16 computes -hi * 1 + v from the f16 half of
// the packed hi word, with one rounding to f16 (v - hi is exact in fp32, so this equals the
// cvt(sub) sequence bit for bit).
__device__ __forceinline__ uint32_t h3_lo_pair(uint32_t hi, float v0, float v1) {
    uint32_t d;
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, -%1, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(d)
        : "v"(hi), "v"(v0), "v"(v1));
    return d;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
// FIRST (the first layer): no residual, keep the result (the first block's skip). RES (the convs,
// in pairs: the block parity is compile-time): 0 = small block 1 (conv + BN + ReLU), 1 = small block
// 2 (conv + BN, + the residual, ReLU; the result is the next block's skip).
template <bool FIRST, bool BF, int RES>
__device__ __forceinline__ void h3t_pack_one(const f32x4& acc, uint32_t (&pk)[2][2], const f32x4& bb, const f32x4& sc,
                                             f32x4& skip) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const f32x2 a2 = {acc[2 * k], acc[2 * k + 1]}, s2 = {sc[2 * k], sc[2 * k + 1]};
        const f32x2 b2 = {bb[2 * k], bb[2 * k + 1]};
        f32x2 v = __builtin_elementwise_fma(a2, s2, b2);
        if constexpr (!FIRST && RES == 1) v += f32x2{skip[2 * k], skip[2 * k + 1]};
        v[0] = v[0] > 0.0f ? v[0] : 0.0f;
        v[1] = v[1] > 0.0f ? v[1] : 0.0f;
        if constexpr (FIRST || RES == 1) {
            skip[2 * k] = v[0];
            skip[2 * k + 1] = v[1];
        }
        if constexpr (BF) {  // one bf16 piece (RNE), no range limit below fp32's
            pk[0][k] = __builtin_bit_cast(uint32_t, bf16x2{(__bf16)v[0], (__bf16)v[1]});
            pk[1][k] = 0u;
        } else {
            uint32_t hi;  // (RNE; one packed conversion)
            asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(hi) : "v"(v[0]), "v"(v[1]));
            pk[0][k] = hi;
            pk[1][k] = h3_lo_pair(hi, v[0], v[1]);
        }
    }
}
template <class C, int GRP, bool FIRST, int RES>
__device__ __forceinline__ void epilogue_h3t_pack(const f32x4 (&acc)[C::NS], uint32_t (&pk)[C::NS][2][2],
                                                  const f32x4& bb, const f32x4& sc, f32x4 (&skip)[C::NS],
                                                  uint32_t& hmax) {
#pragma unroll
    for (int j = 0; j < grp_n(GRP); ++j) {
        h3t_pack_one<FIRST, (bool)C::BF, RES>(acc[j], pk[j], bb, sc, skip[j]);
        // the range guard: both hi pairs of the square in one v_pk_maximum3_f16 (IEEE maximum: an
        // overflowed hi is +inf = 0x7C00, a NaN stays NaN; hi >= +0 after ReLU)
        if constexpr (!C::BF)
            hmax = __builtin_bit_cast(
                uint32_t, __builtin_elementwise_maximum(
                              __builtin_elementwise_maximum(__builtin_bit_cast(f16x2, hmax), __builtin_bit_cast(f16x2, pk[j][0][0])),
                              __builtin_bit_cast(f16x2, pk[j][0][1])));
    }
}
template <class C, int GRP>
__device__ __forceinline__ void epilogue_h3t_store(const uint32_t (&pk)[C::NS][2][2], char* img, int eo) {
#pragma unroll
    for (int j = 0; j < grp_n(GRP); ++j) {
        char* d = img + grp_sq(GRP, j) * (nn::kSB * h3::kRowB) + eo;
        *reinterpret_cast<uint2*>(d) = uint2{pk[j][0][0], pk[j][0][1]};
        if constexpr (!C::BF) *reinterpret_cast<uint2*>(d + h3::kPlaneB) = uint2{pk[j][1][0], pk[j][1][1]};
    }
}

// The whole forward for the waves of square group GRP.
// k_nn_h3 (TR) first layer, all on fp16 MFMA (conv_init_1, net.rs:16-27 / 119-131): for output square
// sq the K dimension is (plane q, tap t) of the 4 bitboard planes and the 17 constant planes (the
// mover's two cards and the colour plane, common.rs:26-80, summed over sq's on-board taps on the
// host: T[sq]). Block 0 = taps 0-7 of plane q (k = 8q + t), block 1 = tap 8 of plane q (k = 32 + 8q)
// and the constant planes (k = 32 + 8q + 1..7). A = weights (hi / lo of s * W), B = the 0/1 inputs,
// exact in fp16: 4 MFMAs of 16 cycles per square instead of 9 fp32 16x16x4 MFMAs of 32 cycles. The
// lane's 8 tap bits of block 0 are three 3-bit row fields of its plane's bitboard (rows of the board
// are 5 contiguous bits, bit of square i = 1 << (31 - i)), gathered into an 8-bit index (board-edge
// masks are compile-time per square) that selects the f16x8 operand from an LDS table.
template <int SQ>
__device__ __forceinline__ uint32_t l1_pattern(uint32_t bb) {
    constexpr int r = SQ / 5, c = SQ % 5;
    // index bits: 0 = tap 2, 1 = tap 1, 2 = tap 0, 3 = tap 5, 4 = tap 4, 5 = tap 3, 6 = tap 7, 7 = tap 6
    uint32_t a = 0, d = 0;
    if constexpr (r > 0) a = (bb >> (35 - SQ)) & 7u;  // squares SQ-6, SQ-5, SQ-4 (bits 2, 1, 0)
    const uint32_t m = (bb >> (30 - SQ)) & 7u;        // SQ-1, SQ, SQ+1
    if constexpr (r < 4) d = (bb >> (26 - SQ)) & 3u;  // SQ+4, SQ+5 (bits 1, 0)
    const uint32_t idx = a | (m << 3) | (d << 6);
    constexpr uint32_t mask = (c == 0 ? ~0xA4u : ~0u) & (c == 4 ? ~0x09u : ~0u) & 0xFFu;
    return idx & mask;
}
template <int SQ>
__device__ __forceinline__ uint32_t l1_tap8(uint32_t bb) {  // square SQ+6 (tap 8) as an fp16 0 / 1.0
    if constexpr (SQ / 5 == 4 || SQ % 5 == 4) return 0u;
    else return ((bb >> (25 - SQ)) & 1u) ? 0x3C00u : 0u;
}
__device__ __forceinline__ void l1_lut_build(char* lut, int tid) {  // entry P, element t: bit pos(t) of P
    constexpr int pos[8] = {2, 1, 0, 5, 4, 3, 7, 6};
    const int P = tid >> 1, h = tid & 1;
    uint32_t w[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int t0 = 4 * h + 2 * k;
        w[k] = (((P >> pos[t0]) & 1) ? 0x3C00u : 0u) | (((P >> pos[t0 + 1]) & 1) ? 0x3C000000u : 0u);
    }
    *reinterpret_cast<uint2*>(lut + P * 16 + h * 8) = uint2{w[0], w[1]};
}
// K block 1 of square sq depends on sq only through its on-board tap set (the constant planes'
// table T[sq] sums over those taps; tap 8's weights are square-independent): 9 classes (corner,
// edge and interior rows x columns). A wave loads each of its classes once.
constexpr int l1_cls(int sq) {
    const int r = sq / 5, c = sq % 5;
    return (r == 0 ? 0 : r == 4 ? 2 : 1) * 3 + (c == 0 ? 0 : c == 4 ? 2 : 1);
}
struct L1Slots {
    int n;
    int8_t slot[25];  // group square j -> its class slot
    int8_t rep[9];    // class slot -> a square of that class (whose K block 1 is loaded)
};
constexpr L1Slots l1_slots(int grp) {
    L1Slots S{};
    int cls[9] = {};
    for (int j = 0; j < grp_n(grp); ++j) {
        const int c = l1_cls(grp_sq(grp, j));
        int k = 0;
        while (k < S.n && cls[k] != c) ++k;
        if (k == S.n) {
            cls[S.n] = c;
            S.rep[S.n] = (int8_t)grp_sq(grp, j);
            ++S.n;
        }
        S.slot[j] = (int8_t)k;
    }
    return S;
}
template <int GRP>
struct L1SlotsOf {
    static constexpr L1Slots S = l1_slots(GRP);
};
template <class F, int... K>
__device__ __forceinline__ void l1_for_slots(F&& f, std::integer_sequence<int, K...>) {
    (f(std::integral_constant<int, K>{}), ...);
}
template <int GRP>
struct L1H {  // the first layer's A operands (K block 0, and K block 1 of each class the wave touches)
    f16x8 a0h, a0l;
    f16x8 a1[L1SlotsOf<GRP>::S.n][2];
};
// issued at kernel start, so the loads overlap the state load, the LUT build and the barrier
template <int GRP>
__device__ __forceinline__ void first_layer_h3f_fetch(L1H<GRP>& R, const float* l1c, int lane, int nt) {
    X6W A;
    A.r = __builtin_amdgcn_make_buffer_rsrc((void*)l1c, (short)0, (int)(26 * h3::kL1Frag * 4), 0x00020000);
    A.voff = (nt * 64 + lane) * 16;
    auto ld = [&](int blk, int pc) {  // [blk][pc][nt][lane]
        return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(A.r, A.voff, (blk * 2 + pc) * 4 * 64 * 16, 0));
    };
    R.a0h = ld(0, 0);
    R.a0l = ld(0, 1);
    constexpr L1Slots S = L1SlotsOf<GRP>::S;
    l1_for_slots(
        [&](auto kc) {
            constexpr int k = decltype(kc)::value;
            R.a1[k][0] = ld(1 + S.rep[k], 0);
            R.a1[k][1] = ld(1 + S.rep[k], 1);
        },
        std::make_integer_sequence<int, S.n>{});
}
template <class C, int GRP, int... J>
__device__ __forceinline__ void first_layer_h3f(f32x4 (&acc)[C::NS], const L1H<GRP>& R, uint32_t bb, int cinfo,
                                                int lane, const char* lds, std::integer_sequence<int, J...>) {
    const int q = lane >> 4;
    constexpr L1Slots S = L1SlotsOf<GRP>::S;
    const f16x8 &a0h = R.a0h, &a0l = R.a0l;
    const auto& a1 = R.a1;
    // block 1 constants: element e >= 1 of quarter q is constant plane c = 7q + e - 1
    const int c0 = cinfo & 15, c1 = (cinfo >> 4) & 15, blue = (cinfo >> 8) & 1;
    uint32_t kw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t v = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int e = 2 * w + h, c = 7 * q + e - 1;
            const bool one = e > 0 && (c < 16 ? (c == c0 || c == c1) : (c == 16 && blue));
            v |= one ? (0x3C00u << (16 * h)) : 0u;
        }
        kw[w] = v;
    }
    const char* lut = lds + h3::kLutOff;
    auto sq_mfma = [&](auto jc) {
        constexpr int j = decltype(jc)::value, sq = grp_sq(GRP, j);
        const f16x8 b0 = *reinterpret_cast<const f16x8*>(lut + l1_pattern<sq>(bb) * 16);
        uint4 w1 = uint4{kw[0] | l1_tap8<sq>(bb), kw[1], kw[2], kw[3]};
        const f16x8 b1 = __builtin_bit_cast(f16x8, w1);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, b0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0l, b0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[S.slot[j]][0], b1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[S.slot[j]][1], b1, acc[j], 0, 0, 0);
    };
    (sq_mfma(std::integral_constant<int, J>{}), ...);
}

// heads (k_nn_h3): the value / policy 1x1 convs as split MFMAs on the LDS image (one 16x16
// tile per square: rows = positions, columns 0 / 1 / 2 = value, policy planes 0 / 1, each scaled by a
// power of two), then the MLPs per position from a feature table in LDS. p: the head parameters
// (after the convs).
template <class C>
__device__ __forceinline__ void h3_heads(const float* p, char* img, const int (&lo)[2], int wave, int lane, int b0,
                                         int B, float* __restrict__ policy, float* __restrict__ value) {
    const int i = lane & 15, kq = lane >> 4;
    {
        const float* hp = p + nn::kValueF + nn::kPolicyF;
        const f16x8* HB = reinterpret_cast<const f16x8*>(hp);
        f16x8 hb[2][2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int pc = 0; pc < 2; ++pc) hb[m][pc] = HB[(C::BF ? m : m * 2 + pc) * 64 + lane];  // BF: [m][lane]
        const float hs = C::BF ? 1.0f : hp[2 * 2 * 64 * 4 + (i < 3 ? i : 0)];
        // MLP weights in flight during the head convs (after hb: vmcnt is in order)
        HeadMM hm;
        heads_mm_fetch(hm, p, wave, lane);
        constexpr int kSqPerWave = (25 + C::WAVES - 1) / C::WAVES;
        f32x4 hacc[kSqPerWave];
#pragma unroll
        for (int q = 0; q < kSqPerWave; ++q) {
            hacc[q] = f32x4{};
            const int sq = wave + q * C::WAVES;
            if (sq < 25) {
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const char* a = img + sq * (nn::kSB * h3::kRowB) + lo[m];
                    const f16x8 ah = *reinterpret_cast<const f16x8*>(a);
                    if constexpr (C::BF) {
                        hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, hb[m][0]), hacc[q], 0, 0, 0);
                        continue;
                    }
                    const f16x8 al = *reinterpret_cast<const f16x8*>(a + h3::kPlaneB);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, hb[m][0], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, hb[m][0], hacc[q], 0, 0, 0);
                    hacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, hb[m][1], hacc[q], 0, 0, 0);
                }
            }
        }
        __syncthreads();  // the image is no longer read: its first 4.8 KB become the feature table
        float* feat = reinterpret_cast<float*>(img);  // [16 positions][80]
        const float hbias = i == 0 ? p[64] : i == 1 ? p[nn::kValueF + 128] : p[nn::kValueF + 129];
#pragma unroll
        for (int q = 0; q < kSqPerWave; ++q) {
            const int sq = wave + q * C::WAVES;
            if (sq < 25 && i < 3)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = __builtin_fmaf(hacc[q][r], hs, hbias);
                    feat[(kq * 4 + r) * 80 + i * 25 + sq] = v > 0.0f ? v : 0.0f;
                }
        }
        __syncthreads();
        heads_mm(hm, feat, feat + nn::kSB * 80, wave, lane, b0, B, policy, value);
    }
}

// The whole forward for the waves of square group GRP. Returns true in a lane that split an
// activation beyond the fp16 range (an fp16 hi term that overflowed, or would have): the tile's
// results are then invalid and k_nn_h3 recomputes them.
// opaque: 0; from an asm statement when the body sits in a loop (k_search_grp), so that its lane offsets
// are not hoisted out of the loop (see nn_h3s_body)
template <class C, int GRP>
__device__ __forceinline__ bool nn_h3_body(const oaz_state* __restrict__ states, const TileSpan sp,
                                           const float* __restrict__ blob, int blocks, float* __restrict__ policy,
                                           float* __restrict__ value, float* lds, int opaque = 0) {
    const int B = sp.end;
    constexpr int NS = C::NS;
    char* img = reinterpret_cast<char*>(lds);
    const int tid = (int)threadIdx.x + opaque, wave = tid >> 6, lane = tid & 63;
    const int nt = wave & 3;
    const int b0 = sp.b0;
    // (bf16 mode with two image buffers: one piece plane each, so the image area is kImageB as well)
    int* pinfo = reinterpret_cast<int*>(lds + (C::BF && !OAZ_H1_PP ? h3::kPlaneB : h3::kImageB) / 4);
    const int i = lane & 15, kq = lane >> 4;
    const int lo[2] = {h3::chunk_off(i, kq), h3::chunk_off(i, 4 + kq)};
    const int cq = nt * 16 + 4 * kq;  // this lane's 4 channels cq .. cq + 3 of position i
    const int eot = h3::chunk_off(i, cq >> 3) + (cq & 7) * 2;

    f32x4 acc[NS];
    f32x4 skip[NS];
    f16x8 bpre[2];  // the next conv's first B pieces (h3_first_b)
    uint32_t hmax = 0;  // largest hi bit patterns (two u16 halves)
    // DBG 2: first layer (MFMA tail + epilogue), conv, barrier 1, epilogue, barrier 2, heads, kernel start (state,
    // LUT, barrier), first-layer MFMAs (incl. their operand loads)
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tm = C::DBG == 2 ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) {
        if constexpr (C::DBG == 2) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph[k] += t - tm;
            tm = t;
        }
    };
    {  // encoder + first layer
        L1Regs<GRP> l1;
        L1H<GRP> l1h;
        // the fp16 first layer's fragments and inverse scales (after the heads; bf16 mode: same section)
        constexpr bool kF16 = !C::BF || OAZ_H1_L1F16;
        const float* l1c = C::BF ? blob + nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (nn::kW64h + nn::kCh) +
                                       nn::kValueF + nn::kPolicyF + 2 * 64 * 4
                                 : blob + nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh) +
                                       nn::kValueF + nn::kPolicyF + h3::kHeadB;
        // the state loads first: vmcnt retires in issue order, so the pinfo / LUT work before the
        // barrier then waits for these and not for the first-layer operands issued after them
        const int b = min(b0 + i, sp.cap - 1);  // an empty tile of a bucket starts past cap
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&states[b]);
        const uint32_t bb = kq == 0 ? w[2] : kq == 1 ? w[0] : kq == 2 ? w[3] : w[1];
        oaz_state st{};
        if (tid < nn::kSB) st = states[b];
        if constexpr (kF16)
            first_layer_h3f_fetch<GRP>(l1h, l1c, lane, nt);
        else
            first_layer_x6_fetch<GRP>(l1, blob, lane, nt);
        if (tid < nn::kSB) {
            const int blue = st.to_move & 1;
            const int c0 = (blue ? st.cards[2] : st.cards[0]) & 15, c1 = (blue ? st.cards[3] : st.cards[1]) & 15;
            pinfo[tid] = c0 | (c1 << 4) | (blue << 8);
        }
        if constexpr (kF16)
            for (int t = tid; t < 512; t += 64 * C::WAVES) l1_lut_build(img + h3::kLutOff, t);
        const f32x4 bias1t = *reinterpret_cast<const f32x4*>(blob + nn::kL1B + cq);
        if (b0 >= B) return false;  // an empty tile of a compacted bucket (uniform over the workgroup)
        __syncthreads();
        stamp(6);
#pragma unroll
        for (int j = 0; j < NS; ++j) acc[j] = skip[j] = f32x4{};
        if constexpr (kF16)  // fp16 MFMA on the 0/1 inputs
            first_layer_h3f<C, GRP>(acc, l1h, bb, pinfo[i], lane, reinterpret_cast<const char*>(lds),
                                    std::make_integer_sequence<int, grp_n(GRP)>{});
        else  // exact fp32 MFMA on the 0/1 inputs, as k_nn_x6
            first_layer_x6<C, GRP>(acc, l1, blob + nn::kL1B + nn::kCh, bb, pinfo[i], lane, nt);
        if constexpr (C::DBG == 2) {  // the MFMA results, so the stamp follows the MFMAs
            float z = 0.0f;
#pragma unroll
            for (int j = 0; j < NS; ++j) z += acc[j][0];
            asm volatile("" ::"v"(z));
        }
        stamp(7);
        uint32_t pk[NS][2][2];
        const f32x4 inv1 = !kF16 ? f32x4{1.0f, 1.0f, 1.0f, 1.0f}
                                 : *reinterpret_cast<const f32x4*>(l1c + 26 * h3::kL1Frag + cq);
        epilogue_h3t_pack<C, GRP, true, 0>(acc, pk, bias1t, inv1, skip, hmax);
        if constexpr (h3_pf<C>()) {
            constexpr size_t kWc = C::BF ? nn::kW64h : h3::kW;
            h3_first_b<C, GRP>(bpre, h3_w(blob + nn::kL1B + nn::kCh + nn::kL1Table, lane, nt, (int)(kWc * 4)));
        }
        epilogue_h3t_store<C, GRP>(pk, img, eot);
        __syncthreads();
    }
    // the 2 * blocks convs in pairs, so the residual's role is compile-time (small block 1: conv + BN +
    // ReLU; small block 2: conv + BN, + skip, ReLU, the result kept as the next skip)
    stamp(0);
    const float* p = blob + nn::kL1B + nn::kCh + nn::kL1Table;
    auto conv_one = [&](auto res, bool more) {
        constexpr int RES = decltype(res)::value;
        constexpr size_t kWc = C::BF ? nn::kW64h : h3::kW;  // B fragments of one conv
        const f32x4 bbt = *reinterpret_cast<const f32x4*>(p + kWc + cq);  // in flight during the conv
        const f32x4 sct = C::BF ? f32x4{1.0f, 1.0f, 1.0f, 1.0f} : *reinterpret_cast<const f32x4*>(p + kWc + nn::kCh + cq);
#pragma unroll
        for (int j = 0; j < NS; ++j) acc[j] = f32x4{};
        // bf16 mode, two buffers: the pair's first conv reads buffer 0 and writes buffer 1, the second
        // reads 1 and writes 0 (the first layer and the heads use buffer 0). Every wave has finished
        // reading the buffer a conv writes before the previous conv's closing barrier, so the
        // in-place barrier between the MFMAs and the stores is not needed.
        constexpr bool kPP = C::BF && OAZ_H1_PP;
        char* const rd = kPP && RES == 1 ? img + h3::kPlaneB : img;
        char* const wr = kPP && RES == 0 ? img + h3::kPlaneB : img;
        conv_h3_run<C, GRP>(acc, rd, h3_w(p, lane, nt, (int)(kWc * 4)), lo, bpre,
                            std::make_integer_sequence<int, H3P<C, GRP>::P.nbat>{});
        stamp(1);
        const float* pc = p;
        p += C::BF ? nn::kW64h + nn::kCh : h3::kW + 2 * nn::kCh;
        uint32_t pk[NS][2][2];
        epilogue_h3t_pack<C, GRP, false, RES>(acc, pk, bbt, sct, skip, hmax);  // before the barrier: a
        // (unconditional, so that the old pieces are dead during the conv; the last conv reloads its own)
        if constexpr (h3_pf<C>()) h3_first_b<C, GRP>(bpre, h3_w(more ? p : pc, lane, nt, (int)(kWc * 4)));
        stamp(3);                                                             // wave done early packs
        if constexpr (!kPP) __syncthreads();                                  // beside its partner's MFMAs
        stamp(2);
        epilogue_h3t_store<C, GRP>(pk, wr, eot);
        stamp(3);
        __syncthreads();
        stamp(4);
    };
    for (int c = 0; c < blocks; ++c) {
        conv_one(std::integral_constant<int, 0>{}, true);
        conv_one(std::integral_constant<int, 1>{}, c + 1 < blocks);
    }
    h3_heads<C>(p, img, lo, wave, lane, b0, B, policy, value);
    if constexpr (C::DBG == 2) {
        stamp(5);
        __syncthreads();
        float v = 0.0f;  // (compile-time indices: the sums stay in scalar registers)
#pragma unroll
        for (int k = 0; k < 8; ++k) v = lane == k ? (float)ph[k] : v;
        if (lane < 8 && b0 + nn::kSB <= B) policy[(size_t)b0 * 50 + wave * 8 + lane] = v;
    }
    if constexpr (C::BF) return false;  // bf16 pieces have fp32's exponent range
    return (hmax & 0xffffu) >= 0x7C00u || (hmax >> 16) >= 0x7C00u;  // hi = inf
}

// fp16-range fallback: a workgroup in which any lane split an activation beyond the fp16 range
// recomputes its 16 positions with the k_nn_x6 body (the exact three-term bf16 split: fp32's
// exponent range, the same fp32-level error) from the OAZ_FP32_SPLIT blob `xblob`, in the same
// launch, and counts the tile in *fallback. Results are therefore never silently wrong and no run
// dies on a range trip; the common path pays one __syncthreads_or at the end of the workgroup
// (the LDS is released only when every wave is done anyway). x6's LDS image (157.7 KB) bounds the
// kernel's LDS; h3's 106.5 KB already allowed one workgroup per CU only, so occupancy is unchanged.
template <class C>
struct H3Fallback {
    static constexpr bool kOn = !C::BF && C::DBG == 0;
    using X = X6Cfg<>;
    // bf16 mode keeps two buffers of one piece plane (+ the position info): 103 KB, and 168 VGPRs, so
    // two tree-kernel waves (80 VGPRs, 15.6 KB per workgroup) fit beside the two NN waves of a SIMD
    static constexpr int kBase = C::BF && !OAZ_H1_L1F16 ? (OAZ_H1_PP ? h3::kImageB : h3::kPlaneB) / 4 + 256
                                                        : h3::kLdsFloats + h3::kLutB / 4;
    static constexpr int kLds = kOn && x6::kLdsFloats > kBase ? x6::kLdsFloats : kBase;
};

// Out of line, so that the fallback's register allocation (k_nn_x6 spills a few VGPRs at 8 waves)
// cannot touch the k_nn_h3 body's: the call is the rare path.
template <class X, int GRP>
__device__ __noinline__ void nn_h3_fallback(const oaz_state* __restrict__ states, const TileSpan sp,
                                            const float* __restrict__ xblob,
                                            int blocks, float* __restrict__ policy, float* __restrict__ value,
                                            float* lds) {
    nn_x6_body<X, GRP>(states, sp, xblob, blocks, policy, value, lds);
}

template <class C>
__global__ void __launch_bounds__(64 * C::WAVES) k_nn_h3(const oaz_state* __restrict__ states, int B,
                                                        const float* __restrict__ blob, int blocks,
                                                        float* __restrict__ policy, float* __restrict__ value,
                                                        const float* __restrict__ xblob,
                                                        unsigned long long* __restrict__ fallback, TileMap tm) {
    __shared__ __attribute__((aligned(16))) float lds[H3Fallback<C>::kLds];
    // DBG 5 (timing only): the workgroup's start / end on the constant 100 MHz clock and its CU
    const uint64_t rt0 = C::DBG == 5 ? __builtin_amdgcn_s_memrealtime() : 0;
    const TileSpan sp = tile_span(tm, B);
    bool ovf;
    const bool g0 = (threadIdx.x >> 8) == 0;  // waves 0-3: square group GRP0 (17 / 15 squares), 4-7: GRP1
    if (g0) {
        __builtin_amdgcn_s_setprio(1);  // (priority to the smaller group measured 6 % slower)
        ovf = nn_h3_body<C, C::GRP0>(states, sp, blob, blocks, policy, value, lds);
    } else {
        ovf = nn_h3_body<C, C::GRP1>(states, sp, blob, blocks, policy, value, lds);
    }
    if constexpr (H3Fallback<C>::kOn) {
        using X = typename H3Fallback<C>::X;
        if (__syncthreads_or(ovf)) {  // uniform over the workgroup; also the barrier before LDS reuse
            if (g0)
                nn_h3_fallback<X, X::GRP0>(states, sp, xblob, blocks, policy, value, lds);
            else
                nn_h3_fallback<X, X::GRP1>(states, sp, xblob, blocks, policy, value, lds);
            if (threadIdx.x == 0) atomicAdd(fallback, 1ull);
        }
    }
    if constexpr (C::DBG == 5) {
        __syncthreads();  // every wave is done
        if (threadIdx.x == 0 && sp.b0 < sp.end) {
            const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
            uint32_t* o = reinterpret_cast<uint32_t*>(policy + (size_t)sp.b0 * 50);
            o[0] = (uint32_t)rt0;
            o[1] = (uint32_t)(rt0 >> 32);
            o[2] = (uint32_t)rt1;
            o[3] = (uint32_t)(rt1 >> 32);
            o[4] = hw;
            o[5] = xcc;
        }
    }
}

// ---- small batches: one position per workgroup (k_nn_h3s, OAZ_FP32_SPLIT16) ---------------------------
// k_nn_h3 evaluates 16 positions per workgroup (square-major tiles), so below ~16 x 256 positions a
// launch leaves CUs idle and a single position (the Agent API's generate_move, alphazero_mcts/mod.rs:
// 122-144; an arena's last games, evaluator.rs:355-399) still costs a whole 16-position workgroup
// lifetime (~60-70 us). Here a workgroup evaluates ONE position: the GEMM columns are the position's
// squares (two 16-column tiles, 25 of 32 used).
// The arithmetic is k_nn_h3's, element for element, so the two kernels give bit-identical outputs
// (the tree-parity tests rely on the network being batch-independent): the same packed fp16 hi/lo
// weights as the MFMA A operand, the image as B with the same channel-to-k mapping, per output element
// the same MFMA sequence (steps = (tap, K-half) in order, each lo*hi, hi*hi, hi*lo) — a (square, tap)
// that k_nn_h3 skips because the neighbour is off the board reads the zero row here and adds an exact
// +-0 — the same epilogue (fma(acc, 1/s, bias), residual, ReLU, RNE hi / exact lo split), the same
// first-layer K blocks (the square-class-dependent K block 1 is applied once per class present in
// the tile, with the B columns of the other classes zeroed), the same head 1x1-conv MFMAs and heads_mm.
// The fp16-range guard and its in-kernel recompute (the k_nn_x6 body for this position) are k_nn_h3's.
// Bound: one position's weights (147 KB of fp16 hi/lo per 3x3 conv) through ONE CU's vector memory
// path (~64 B/clk), not the MFMAs (1.7k cycles per conv per SIMD). So every conv weight is fetched
// once per workgroup: waves 0-3 (one per SIMD) own an N-tile (16 output channels) and BOTH column
// tiles (two independent accumulators share each weight fragment), keep a conv's 18 (tap, K-half)
// steps x 2 pieces in registers (144 VGPRs) and request the next conv's step by step as this conv
// retires them. Waves 4-7 take what would sit on that path's critical start and end: the first layer
// (its fp32 results go to the compute waves through LDS as the first block's residual) and the heads'
// 1x1 convs, their weights requested at kernel start. The image is two 26-row buffers (ping-pong: one
// barrier per conv) with a zero row for off-board taps. 8 waves also make the k_nn_x6 fallback body
// (8 waves) callable in the same launch.
namespace h3s {
constexpr int kRows = 26;  // 25 squares + the zero row
constexpr int kZero = 25;
constexpr int kRowB = 128;                  // one piece: 64 channels x f16
constexpr int kPlaneB = kRows * kRowB;      // 3,328 B
constexpr int kImageB = 2 * kPlaneB;        // hi + lo pieces
constexpr int kSkipOff = 2 * kImageB;       // two image buffers, then the first layer's fp32 results:
                                            // [4 N-tiles][64 lanes][2 tiles] f32x4
constexpr int kHeadOff = kSkipOff + 4 * 64 * 2 * 16;  // the head parameters (value, policy, head 1x1 B pieces)
constexpr int kHeadF = (int)(nn::kValueF + nn::kPolicyF + h3::kHeadB);  // 5,512 floats
constexpr int kFeatOff = kHeadOff + ((kHeadF * 4 + 15) & ~15);  // features [16][80] + heads_mm's table [16][128]
constexpr int kBytes = kFeatOff + (16 * 80 + 16 * 128) * 4;
// 16-byte chunk c8 of a row at c8 ^ (row & 7): the 16 rows a 16-lane group reads spread over the banks
__device__ __forceinline__ int chunk_off(int row, int c8) { return row * kRowB + ((c8 ^ (row & 7)) << 4); }
}  // namespace h3s

// l1_pattern / l1_tap8 for a run-time square (here a lane's column is a square, not a position)
__device__ __forceinline__ uint32_t l1_pattern_rt(int sq, uint32_t bb) {
    const int r = sq / 5, c = sq % 5;
    const uint32_t a = r > 0 ? (bb >> (35 - sq)) & 7u : 0u;
    const uint32_t m = (bb >> (30 - sq)) & 7u;
    const uint32_t d = r < 4 ? (bb >> (26 - sq)) & 3u : 0u;
    const uint32_t mask = (c == 0 ? ~0xA4u : ~0u) & (c == 4 ? ~0x09u : ~0u) & 0xFFu;
    return (a | (m << 3) | (d << 6)) & mask;
}
// l1_lut_build's entry for pattern P, built in registers: element t = bit pos(t) of P as fp16 0 / 1.0
__device__ __forceinline__ f16x8 l1_pattern_frag(uint32_t P) {
    constexpr int pos[8] = {2, 1, 0, 5, 4, 3, 7, 6};
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w[k] = (((P >> pos[2 * k]) & 1u) ? 0x3C00u : 0u) | (((P >> pos[2 * k + 1]) & 1u) ? 0x3C000000u : 0u);
    return __builtin_bit_cast(f16x8, uint4{w[0], w[1], w[2], w[3]});
}
__device__ __forceinline__ uint32_t l1_tap8_rt(int sq, uint32_t bb) {
    if (sq / 5 == 4 || sq % 5 == 4) return 0u;
    return ((bb >> (25 - sq)) & 1u) ? 0x3C00u : 0u;
}
__device__ __forceinline__ int l1_cls_rt(int sq) {
    const int r = sq / 5, c = sq % 5;
    return (r == 0 ? 0 : r == 4 ? 2 : 1) * 3 + (c == 0 ? 0 : c == 4 ? 2 : 1);
}
// a representative square of each first-layer class (whose K block 1 is loaded)
__constant__ int8_t c_cls_rep[9] = {0, 1, 4, 5, 6, 9, 20, 21, 24};

struct H3sW {  // one conv's B pieces: 18 steps x (hi, lo)
    f16x8 w[18][2];
};
// byte offset of the B fragment (K-half m) of square sq's neighbour for tap t: the zero row when it is
// off the board or sq is a padding column
__device__ __forceinline__ int h3s_boff(int sq, int t, int m, int kq) {
    const int row = sq < 25 ? nbr_index(sq, t) : h3s::kZero;  // nbr_index: 25 = off the board
    return h3s::chunk_off(row, 4 * m + kq);
}

// Operands the one-launch search (k_search_lat) keeps resident in LDS across its simulations (loaded
// once per launch, again after an fp16-range recompute, which uses the whole LDS): the first layer's
// K blocks (block 0 and one block-1 per square class: [10][2 pieces][4 N-tiles][64 lanes] f16x8), its
// bias and inverse scales, and the head parameters; and the leaf position, written there by the walk.
namespace h3s {
constexpr int kL1Off = kBytes;                      // after the body's own LDS
constexpr int kL1Bytes = 10 * 2 * 4 * 64 * 16;      // 80 KB
constexpr int kL1BiasOff = kL1Off + kL1Bytes;       // bias1[64], inv1[64]
constexpr int kStateOff = kL1BiasOff + 2 * 64 * 4;  // the leaf position (24 B)
constexpr int kResidentBytes = kStateOff + 32;
}  // namespace h3s
struct H3sResident {
    const oaz_state* state;  // LDS: the position to evaluate (null: states[b])
    const char* l1;          // LDS: kL1Bytes of first-layer fragments + bias / inverse scales (null: global)
    bool heads;              // the head parameters are already in the body's LDS (no copy)
};
// opaque: 0, produced by an asm statement when the body sits in a loop (k_search_lat), so that the
// lane-dependent offsets are computed where they are used instead of being hoisted out of the loop and
// kept live through the convs (which then spill)
template <class C>
__device__ __forceinline__ bool nn_h3s_body(const oaz_state* __restrict__ states, int b, const float* __restrict__ blob,
                                            int blocks, float* __restrict__ policy, float* __restrict__ value,
                                            float* lds, int opaque = 0, H3sResident res = H3sResident{nullptr, nullptr, false}) {
    static_assert(!C::BF && C::WAVES == 8, "k_nn_h3s: fp16x3 mode, 8 waves");
    // DBG 2 (diagnostic build, timing only): per-wave s_memtime phase sums over the position's policy row:
    // 0 kernel start to the first conv (helpers: the first layer), 2 conv MFMA loops, 3 conv epilogues +
    // barriers, 4 heads 1x1 convs, 5 heads MLP / softmax
    uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tmk = C::DBG == 2 ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) {
        if constexpr (C::DBG == 2) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph[k] += t - tmk;
            tmk = t;
        }
    };
    char* const base = reinterpret_cast<char*>(lds);
    char* const img0 = base;
    char* const img1 = base + h3s::kImageB;
    f32x4* const skipx = reinterpret_cast<f32x4*>(base + h3s::kSkipOff);
    float* const hl = reinterpret_cast<float*>(base + h3s::kHeadOff);  // the head parameters in LDS
    float* const feat = reinterpret_cast<float*>(base + h3s::kFeatOff);
    const int tid = (int)threadIdx.x + opaque, wave = tid >> 6, lane = tid & 63;
    const bool compute = wave < 4;  // waves 0-3: the convs; 4-7: first layer, head parameters, head convs
    const int nt = wave & 3;
    const int i = lane & 15, kq = lane >> 4;
    const int sq0 = i, sq1 = 16 + i;  // the lane's columns in tiles 0 and 1 (sq1 >= 25: padding)
    const bool live1 = sq1 < 25;
    const int cq = nt * 16 + 4 * kq;  // this lane's 4 output channels cq .. cq + 3
    const int eo0 = h3s::chunk_off(sq0, cq >> 3) + (cq & 7) * 2;
    const int eo1 = h3s::chunk_off(live1 ? sq1 : h3s::kZero, cq >> 3) + (cq & 7) * 2;
    const float* l1c = blob + nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh) +
                       nn::kValueF + nn::kPolicyF + h3::kHeadB;
    const float* p = blob + nn::kL1B + nn::kCh + nn::kL1Table;  // the first conv's packed weights
    const float* ph0 = p + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh);  // the head parameters
    uint32_t hmax = 0;
    auto track = [&](const uint32_t (&pk)[2][2]) {  // the fp16 range guard (hi >= +0 after ReLU)
        hmax = __builtin_bit_cast(
            uint32_t, __builtin_elementwise_maximum(
                          __builtin_elementwise_maximum(__builtin_bit_cast(f16x2, hmax), __builtin_bit_cast(f16x2, pk[0][0])),
                          __builtin_bit_cast(f16x2, pk[0][1])));
    };
    auto store2 = [&](char* img, int eo, const uint32_t (&pk)[2][2]) {
        *reinterpret_cast<uint2*>(img + eo) = uint2{pk[0][0], pk[0][1]};
        *reinterpret_cast<uint2*>(img + h3s::kPlaneB + eo) = uint2{pk[1][0], pk[1][1]};
    };
    H3sW R;  // compute waves: the current conv's B pieces
    if (compute) {
        const X6W W0 = h3_w(p, lane, nt);
#pragma unroll
        for (int st = 0; st < 18; ++st) {  // the first conv's pieces, in flight during the first layer
            R.w[st][0] = h3_ldb(W0, (st * 2 + 0) * 4);
            R.w[st][1] = h3_ldb(W0, (st * 2 + 1) * 4);
        }
        if (tid < 32)  // the zero row of both buffers, both pieces (32 x 16 B)
            *reinterpret_cast<uint4*>(base + (tid >> 4) * h3s::kImageB + ((tid >> 3) & 1) * h3s::kPlaneB +
                                      h3s::kZero * h3s::kRowB + (tid & 7) * 16) = uint4{0u, 0u, 0u, 0u};
    } else {  // ---- helpers: the first layer (k_nn_h3's K blocks) for N-tile nt, both tiles; no barrier inside
        const oaz_state st = res.state ? *res.state : states[b];
        f16x8 a0h, a0l, a1[9][2];
        f32x4 bias1t, inv1;
        if (res.l1) {  // resident in LDS: [slot][pc][nt][lane], slot 0 = block 0, 1 + k = class k's block 1
            const f16x8* L = reinterpret_cast<const f16x8*>(res.l1) + nt * 64 + lane;
            a0h = L[0];
            a0l = L[256];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                a1[k][0] = L[((1 + k) * 2 + 0) * 256];
                a1[k][1] = L[((1 + k) * 2 + 1) * 256];
            }
            bias1t = *reinterpret_cast<const f32x4*>(res.l1 + h3s::kL1Bytes + cq * 4);
            inv1 = *reinterpret_cast<const f32x4*>(res.l1 + h3s::kL1Bytes + 256 + cq * 4);
        } else {
            X6W A;
            A.r = __builtin_amdgcn_make_buffer_rsrc((void*)l1c, (short)0, (int)(26 * h3::kL1Frag * 4), 0x00020000);
            A.voff = (nt * 64 + lane) * 16;
            auto ld = [&](int blk, int pc) {  // [blk][pc][nt][lane]
                return __builtin_bit_cast(
                    f16x8, __builtin_amdgcn_raw_buffer_load_b128(A.r, A.voff, (blk * 2 + pc) * 4 * 64 * 16, 0));
            };
            a0h = ld(0, 0);
            a0l = ld(0, 1);
#pragma unroll
            for (int k = 0; k < 9; ++k) {  // every class occurs in one of the two tiles
                a1[k][0] = ld(1 + c_cls_rep[k], 0);
                a1[k][1] = ld(1 + c_cls_rep[k], 1);
            }
            bias1t = *reinterpret_cast<const f32x4*>(blob + nn::kL1B + cq);
            inv1 = *reinterpret_cast<const f32x4*>(l1c + 26 * h3::kL1Frag + cq);
        }
        const uint32_t bb = kq == 0 ? st.pawns[0] : kq == 1 ? st.kings[0] : kq == 2 ? st.pawns[1] : st.kings[1];
        const int blue = st.to_move & 1;
        const int c0 = (blue ? st.cards[2] : st.cards[0]) & 15, c1 = (blue ? st.cards[3] : st.cards[1]) & 15;
        // block 1's constant planes: element e >= 1 of quarter q is constant plane c = 7q + e - 1
        uint32_t kw[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            uint32_t v = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = 2 * w + h, c = 7 * kq + e - 1;
                const bool one = e > 0 && (c < 16 ? (c == c0 || c == c1) : (c == 16 && blue));
                v |= one ? (0x3C00u << (16 * h)) : 0u;
            }
            kw[w] = v;
        }
        const int cls0 = l1_cls_rt(sq0), cls1 = live1 ? l1_cls_rt(sq1) : -1;
        const f16x8 b00 = l1_pattern_frag(l1_pattern_rt(sq0, bb));
        const f16x8 b01 = l1_pattern_frag(live1 ? l1_pattern_rt(sq1, bb) : 0u);
        const f16x8 b10 = __builtin_bit_cast(f16x8, uint4{kw[0] | l1_tap8_rt(sq0, bb), kw[1], kw[2], kw[3]});
        const f16x8 b11 = __builtin_bit_cast(f16x8, uint4{kw[0] | (live1 ? l1_tap8_rt(sq1, bb) : 0u), kw[1], kw[2], kw[3]});
        const f16x8 bz = {};
        f32x4 acc0 = {}, acc1 = {};
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, b00, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, b01, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0l, b00, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0l, b01, acc1, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const f16x8 bk0 = cls0 == k ? b10 : bz, bk1 = cls1 == k ? b11 : bz;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[k][0], bk0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[k][0], bk1, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[k][1], bk0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[k][1], bk1, acc1, 0, 0, 0);
        }
        uint32_t pk[2][2];
        f32x4 r0 = {}, r1 = {};
        h3t_pack_one<true, false, 0>(acc0, pk, bias1t, inv1, r0);
        track(pk);
        store2(img0, eo0, pk);
        h3t_pack_one<true, false, 0>(acc1, pk, bias1t, inv1, r1);
        if (live1) {
            track(pk);
            store2(img0, eo1, pk);
        }
        skipx[(nt * 64 + lane) * 2 + 0] = r0;  // the first block's residual, for the compute waves
        skipx[(nt * 64 + lane) * 2 + 1] = r1;
    }
    __syncthreads();  // the first layer's image and residual
    stamp(0);
    if (!compute && !res.heads) {  // the head parameters into LDS during the first conv (no global round trip at the end)
        static_assert(h3s::kHeadF % 4 == 0, "float4 copy");
        const float4* src = reinterpret_cast<const float4*>(ph0);
        float4* dst = reinterpret_cast<float4*>(hl);
        for (int k = tid - 256; k < h3s::kHeadF / 4; k += 256) dst[k] = src[k];
    }
    f32x4 skip0 = {}, skip1 = {};  // compute waves: the residual (fp32) of both tiles
    if (compute) {
        skip0 = skipx[(nt * 64 + lane) * 2 + 0];
        skip1 = skipx[(nt * 64 + lane) * 2 + 1];
    }
    // the 2 * blocks convs in pairs (compile-time residual role, as k_nn_h3): conv c reads buffer c & 1
    // and writes the other; the helpers only keep the barrier count
    auto conv_one = [&](auto res, bool more, const char* rd, char* wr) {
        constexpr int RES = decltype(res)::value;
        if (compute) {
            const f32x4 bbt = *reinterpret_cast<const f32x4*>(p + h3::kW + cq);
            const f32x4 sct = *reinterpret_cast<const f32x4*>(p + h3::kW + nn::kCh + cq);
            const X6W Wn = h3_w(p + h3::kW + 2 * nn::kCh, lane, nt);
            f32x4 acc0 = {}, acc1 = {};
            f16x8 xl0[2], xh0[2], xl1[2], xh1[2];
            {
                const int o0 = h3s_boff(sq0, 0, 0, kq), o1 = h3s_boff(sq1, 0, 0, kq);
                xl0[0] = *reinterpret_cast<const f16x8*>(rd + h3s::kPlaneB + o0);
                xh0[0] = *reinterpret_cast<const f16x8*>(rd + o0);
                xl1[0] = *reinterpret_cast<const f16x8*>(rd + h3s::kPlaneB + o1);
                xh1[0] = *reinterpret_cast<const f16x8*>(rd + o1);
            }
#pragma unroll
            for (int s = 0; s < 18; ++s) {
                if (s + 1 < 18) {  // the next step's fragments
                    const int t = (s + 1) >> 1, m = (s + 1) & 1, n = (s + 1) & 1;
                    const int o0 = h3s_boff(sq0, t, m, kq), o1 = h3s_boff(sq1, t, m, kq);
                    xl0[n] = *reinterpret_cast<const f16x8*>(rd + h3s::kPlaneB + o0);
                    xh0[n] = *reinterpret_cast<const f16x8*>(rd + o0);
                    xl1[n] = *reinterpret_cast<const f16x8*>(rd + h3s::kPlaneB + o1);
                    xh1[n] = *reinterpret_cast<const f16x8*>(rd + o1);
                }
                const int c = s & 1;
                acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(R.w[s][0], xl0[c], acc0, 0, 0, 0);  // lo * hi
                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(R.w[s][0], xl1[c], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(R.w[s][0], xh0[c], acc0, 0, 0, 0);  // hi * hi
                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(R.w[s][0], xh1[c], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(R.w[s][1], xh0[c], acc0, 0, 0, 0);  // hi * lo
                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(R.w[s][1], xh1[c], acc1, 0, 0, 0);
                if (more) {  // the next conv's step s (uniform branch)
                    R.w[s][0] = h3_ldb(Wn, (s * 2 + 0) * 4);
                    R.w[s][1] = h3_ldb(Wn, (s * 2 + 1) * 4);
                }
            }
            if constexpr (C::DBG == 2) asm volatile("" ::"v"(acc0[0]), "v"(acc1[0]));  // the stamp follows the MFMAs
            stamp(2);
            uint32_t pk[2][2];
            h3t_pack_one<false, false, RES>(acc0, pk, bbt, sct, skip0);
            track(pk);
            store2(wr, eo0, pk);
            h3t_pack_one<false, false, RES>(acc1, pk, bbt, sct, skip1);
            if (live1) {
                track(pk);
                store2(wr, eo1, pk);
            }
        }
        p += h3::kW + 2 * nn::kCh;
        __syncthreads();
        stamp(3);
    };
    for (int c = 0; c < blocks; ++c) {
        conv_one(std::integral_constant<int, 0>{}, true, img0, img1);
        conv_one(std::integral_constant<int, 1>{}, c + 1 < blocks, img1, img0);
    }
    if (blocks == 0) __syncthreads();  // the head parameters' copy (no conv barrier in between)
    // heads (h3_heads' arithmetic, parameters from LDS): the 1x1 convs by waves 4, 5 with the image as A
    // (rows = squares), then heads_mm over all 8 waves
    {
        HeadMM hm;
        heads_mm_fetch(hm, hl, wave, lane);
        const float hs = hl[nn::kValueF + nn::kPolicyF + 2 * 2 * 64 * 4 + (i < 3 ? i : 0)];
        const float hbias = i == 0 ? hl[64] : i == 1 ? hl[nn::kValueF + 128] : hl[nn::kValueF + 129];
        if (wave == 4 || wave == 5) {
            const f16x8* HB = reinterpret_cast<const f16x8*>(hl + nn::kValueF + nn::kPolicyF);
            f16x8 hb[2][2];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int pc = 0; pc < 2; ++pc) hb[m][pc] = HB[(m * 2 + pc) * 64 + lane];
            const int rt = wave - 4;
            const int rsq = rt * 16 + i;  // A row = square
            const int row = rsq < 25 ? rsq : h3s::kZero;
            f32x4 hacc = {};
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const char* a = img0 + h3s::chunk_off(row, 4 * m + kq);
                const f16x8 ah = *reinterpret_cast<const f16x8*>(a);
                const f16x8 al = *reinterpret_cast<const f16x8*>(a + h3s::kPlaneB);
                hacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, hb[m][0], hacc, 0, 0, 0);
                hacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, hb[m][0], hacc, 0, 0, 0);
                hacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, hb[m][1], hacc, 0, 0, 0);
            }
            // C/D: reg r of lane l = (row 4 * kq + r = square rt * 16 + 4 * kq + r, column i = head output)
            if (i < 3)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int s2 = rt * 16 + 4 * kq + r;
                    const float v = __builtin_fmaf(hacc[r], hs, hbias);
                    if (s2 < 25) feat[i * 25 + s2] = v > 0.0f ? v : 0.0f;
                }
        } else {
            const int t0 = compute ? tid : tid - 256 + 128;  // waves 0-3, 6, 7: rows 1-15 (unused positions)
            for (int k = t0; k < 15 * 80; k += 384) feat[80 + k] = 0.0f;
        }
        __syncthreads();
        stamp(4);
        heads_mm(hm, feat, feat + 16 * 80, wave, lane, b, b + 1, policy, value);
    }
    if constexpr (C::DBG == 2) {
        stamp(5);
        __syncthreads();
        float v = 0.0f;
#pragma unroll
        for (int k = 0; k < 6; ++k) v = lane == k ? (float)ph[k] : v;
        if (lane < 6) policy[(size_t)b * 50 + wave * 6 + lane] = v;
    }
    return (hmax & 0xffffu) >= 0x7C00u || (hmax >> 16) >= 0x7C00u;  // an fp16 hi term overflowed
}

// The one-launch search's resident operands (H3sResident): all threads of the workgroup, then a barrier.
__device__ __forceinline__ void h3s_load_resident(char* lds, const float* blob, int blocks) {
    const float* l1c = blob + nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh) +
                       nn::kValueF + nn::kPolicyF + h3::kHeadB;
    const float* ph0 = blob + nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh);
    const int tid = (int)threadIdx.x;
    uint4* d = reinterpret_cast<uint4*>(lds + h3s::kL1Off);
    for (int k = tid; k < h3s::kL1Bytes / 16; k += (int)blockDim.x) {  // [slot][pc][nt][lane]
        const int slot = k / 512, rest = k % 512;
        const int blk = slot == 0 ? 0 : 1 + c_cls_rep[slot - 1];
        d[k] = reinterpret_cast<const uint4*>(l1c)[blk * 512 + rest];
    }
    float* bi = reinterpret_cast<float*>(lds + h3s::kL1BiasOff);
    if (tid < 64) bi[tid] = blob[nn::kL1B + tid];
    else if (tid < 128) bi[tid] = l1c[26 * h3::kL1Frag + tid - 64];
    float4* hd = reinterpret_cast<float4*>(lds + h3s::kHeadOff);
    for (int k = tid; k < h3s::kHeadF / 4; k += (int)blockDim.x) hd[k] = reinterpret_cast<const float4*>(ph0)[k];
    __syncthreads();
}

template <class C>
__global__ void __launch_bounds__(64 * C::WAVES) k_nn_h3s(const oaz_state* __restrict__ states, int B,
                                                         const float* __restrict__ blob, int blocks,
                                                         float* __restrict__ policy, float* __restrict__ value,
                                                         const float* __restrict__ xblob,
                                                         unsigned long long* __restrict__ fallback, TileMap tm) {
    __shared__ __attribute__((aligned(16))) float lds[H3Fallback<C>::kLds];
    static_assert(h3s::kBytes <= H3Fallback<C>::kLds * 4, "k_nn_h3s LDS");
    int b = (int)blockIdx.x, end = B, cap = B;
    if (tm.bcnt) {  // compacted leaves: workgroup i takes row i / nb of bucket i % nb
        const int bk = (int)blockIdx.x % tm.nb;
        b = (bk << kBucketShift) + (int)blockIdx.x / tm.nb;
        end = (bk << kBucketShift) + (int)tm.bcnt[bk];
        cap = tm.cap;
    }
    if (b >= end) return;  // uniform over the workgroup
    const bool ovf = nn_h3s_body<C>(states, b, blob, blocks, policy, value, lds);
    if constexpr (H3Fallback<C>::kOn) {
        using X = typename H3Fallback<C>::X;
        if (__syncthreads_or(ovf)) {  // recompute this position as k_nn_h3 would (its fallback body)
            const TileSpan sp{b, b + 1, cap};
            if ((threadIdx.x >> 8) == 0)
                nn_h3_fallback<X, X::GRP0>(states, sp, xblob, blocks, policy, value, lds);
            else
                nn_h3_fallback<X, X::GRP1>(states, sp, xblob, blocks, policy, value, lds);
            if (threadIdx.x == 0) atomicAdd(fallback, 1ull);
        }
    }
}

// One kernel per precision. The A/B build (make AB=1, -DOAZ_AB=1) adds the diagnostic builds of
// k_nn_h3, selected by OAZ_NN_X6_V (timing only, wrong results); the product build ignores it.
hipError_t launch_nn_forward(const NNView& w, const oaz_state* s, int B, float* policy, float* value,
                             hipStream_t st) {
    if (B <= 0) return hipSuccess;
    // compacted leaves (B = games): as many tiles per bucket as its games could fill (the empty ones
    // exit early); plain: ceil(B / 16)
    const int per_bucket = ((B < (int)kBucket ? B : (int)kBucket) + nn::kSB - 1) / nn::kSB;
    const unsigned grid = w.tm.bcnt ? (unsigned)(w.tm.nb * per_bucket) : (unsigned)((B + nn::kSB - 1) / nn::kSB);
    const dim3 block(64 * nn::kWaves);
    if (w.precision == OAZ_FP32_SPLIT16) {
        if (!w.fallback || !w.blob_x6) return hipErrorInvalidValue;
        if (B <= w.small_max) {  // one position per workgroup (bit-identical results, ~10x less latency)
            const unsigned g1 = w.tm.bcnt ? (unsigned)(w.tm.nb * (B < (int)kBucket ? B : (int)kBucket)) : (unsigned)B;
            auto ks = k_nn_h3s<H3Cfg<0>>;
#if OAZ_AB
            if (w.x6_variant == 70) ks = k_nn_h3s<H3Cfg<0, 2>>;  // phase stamps (timing only)
#endif
            hipLaunchKernelGGL(ks, dim3(g1), block, 0, st, s, B, w.blob, w.blocks, policy, value,
                               w.blob_x6, w.fallback, w.tm);
            return hipGetLastError();
        }
        // 8 waves, uneven 17 / 8 square split, batches of <= 4 squares, transposed C/D tiles, convs in
        // pairs (compile-time residual), in-kernel k_nn_x6 recompute of fp16-range tiles
        auto k = k_nn_h3<H3Cfg<0>>;
#if OAZ_AB
        switch (w.x6_variant) {
            case 36: k = k_nn_h3<H3Cfg<0, 2>>; break;  // phase stamps (tools/nn_phases.py)
            case 40: k = k_nn_h3<H3Cfg<0, 3>>; break;  // ablation: no conv A reads
            case 41: k = k_nn_h3<H3Cfg<0, 4>>; break;  // ablation: no conv B loads
            case 47: k = k_nn_h3<H3Cfg<0, 7>>; break;  // ablation: conv B loads from one step (L1 hits)
            case 49: k = k_nn_h3<H3Cfg<0, 9>>; break;  // ablation: conv A reads discarded (stale operands)
            case 60: k = k_nn_h3<H3Cfg<0, 5>>; break;  // workgroup timeline (tools/nn_timeline.py)
            default: break;
        }
#endif
        hipLaunchKernelGGL(k, dim3(grid), block, 0, st, s, B, w.blob, w.blocks, policy, value, w.blob_x6, w.fallback,
                           w.tm);
    } else if (w.precision == OAZ_FP32_SPLIT) {
        // 8 waves, uneven 15 / 10 square split, pipelined batches of <= 4 squares
        hipLaunchKernelGGL(k_nn_x6<X6Cfg<>>, dim3(grid), block, 0, st, s, B, w.blob, w.blocks, policy, value, w.tm);
    } else if (w.precision == OAZ_BF16) {
        // the k_nn_h3 structure with one bf16 piece and one product, convs in pairs
        hipLaunchKernelGGL(k_nn_h3<H3Cfg<1>>, dim3(grid), block, 0, st, s, B, w.blob, w.blocks, policy, value, nullptr,
                           nullptr, w.tm);
    } else {
        hipLaunchKernelGGL(k_nn_sq16, dim3(grid), block, 0, st, s, B, w.blob, w.blocks, policy, value, w.tm);
    }
    return hipGetLastError();
}

}  // namespace oaz
