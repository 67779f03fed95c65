// pmc_cal.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access shapes of the tree
// kernels (MI355X_MICROARCH.md, HBM: "calibrate on a known byte count in your own access pattern before
// trusting an absolute"). Each kernel touches a known number of bytes, every line once, spread over a 4 GiB
// buffer (far past the 4 MiB L2s and the 256 MiB Infinity Cache) by a multiplicative permutation:
//   k_cal_stream16   16 B per lane, consecutive (the guide's wide streaming read: FETCH_SIZE = 1/2)
//   k_cal_rec32      one 32-byte node per lane (two 16-B loads), random node
//   k_cal_run400     a 16-lane segment reads 400 contiguous bytes (12.5 nodes: a node's children)
//   k_cal_rec24      one 24-byte position per lane (three 8-B loads), random record
//   k_cal_word4      one 4-byte word per lane (a path entry), random 64-B line
//   k_cal_word8      one 8-byte word per lane (sqrt(N), a noise pair), random 64-B line
//   k_cal_coal4      4 B per lane, consecutive (a coalesced 256-B wave read: the BN / reduction kernels)
//   k_cal_seg64      64 B per 4 lanes (16 B each) at a random 64-B line (the conv A fragments' row segments)
//   k_cal_wstream16  16 B per lane written, consecutive
//   k_cal_wrec12     12 bytes per lane written (a node's N and W), random node
//   k_cal_wword4     4 bytes per lane written, random 64-B line
// Build: hipcc --offload-arch=gfx950 -O3 -o pmc_cal pmc_cal.hip; run under
// rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) --kernel-trace-free pass; tools/pmc_cal/analyse.py reads the CSVs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint64_t kBytes = 4ull << 30;
constexpr uint32_t kN = 1u << 22;  // accesses (lanes) per kernel: 4 M

__device__ __forceinline__ uint64_t perm(uint64_t i, uint64_t n) { return (i * 2654435761ull) & (n - 1); }

__global__ void k_cal_stream16(const uint4* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 v = p[i];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = i;
}
__global__ void k_cal_rec32(const uint4* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t r = perm(i, kBytes / 32);
    const uint4 a = p[2 * r], b = p[2 * r + 1];
    if ((a.x ^ b.w) == 0x12345678u) out[0] = i;
}
__global__ void k_cal_run400(const uint4* p, uint32_t* out) {  // 16 lanes x 25 B: 25 x 16 B loads per segment
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, seg = i >> 4, l = i & 15;
    const uint64_t base = perm(seg, kBytes / 512) * 32;  // 512-B slots, 400 B used (uint4 index)
    uint32_t acc = 0;
    for (uint32_t k = l; k < 25; k += 16) acc ^= p[base + k].x;
    if (acc == 0x12345678u) out[0] = i;
}
__global__ void k_cal_rec24(const uint2* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t r = perm(i, kBytes / 32);  // 24-B records at 32-B strides: each record inside one sector
    const uint2 a = p[4 * r], b = p[4 * r + 1], c = p[4 * r + 2];
    if ((a.x ^ b.y ^ c.x) == 0x12345678u) out[0] = i;
}
__global__ void k_cal_word4(const uint32_t* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t v = p[perm(i, kBytes / 64) * 16];
    if (v == 0x12345678u) out[0] = i;
}
__global__ void k_cal_word8(const uint2* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint2 v = p[perm(i, kBytes / 64) * 8];
    if ((v.x ^ v.y) == 0x12345678u) out[0] = i;
}
__global__ void k_cal_coal4(const uint32_t* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t v = p[i];
    if (v == 0x12345678u) out[0] = i;
}
__global__ void k_cal_seg64(const uint4* p, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 v = p[perm(i >> 2, kBytes / 64) * 4 + (i & 3)];
    if ((v.x ^ v.w) == 0x12345678u) out[0] = i;
}
__global__ void k_cal_wstream16(uint4* p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    p[i] = make_uint4(i, i, i, i);
}
__global__ void k_cal_wrec12(uint32_t* p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t* q = p + perm(i, kBytes / 32) * 8 + 4;  // N (4 B) and W (8 B) at bytes 16..27 of a 32-B node
    q[0] = i;
    q[1] = i;
    q[2] = i;
}
__global__ void k_cal_wword4(uint32_t* p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    p[perm(i, kBytes / 64) * 16] = i;
}

int main() {
    void* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    if (hipMemset(buf, 1, kBytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "memset failed\n");
        return 1;
    }
    const dim3 grid(kN / 256), blk(256);
    // read kernels: each launch is preceded by a write pass elsewhere so its lines are not L2-resident
    hipLaunchKernelGGL(k_cal_stream16, grid, blk, 0, 0, (const uint4*)buf, out);
    hipLaunchKernelGGL(k_cal_rec32, grid, blk, 0, 0, (const uint4*)buf, out);
    hipLaunchKernelGGL(k_cal_run400, grid, blk, 0, 0, (const uint4*)buf, out);
    hipLaunchKernelGGL(k_cal_rec24, grid, blk, 0, 0, (const uint2*)buf, out);
    hipLaunchKernelGGL(k_cal_word4, grid, blk, 0, 0, (const uint32_t*)buf, out);
    hipLaunchKernelGGL(k_cal_word8, grid, blk, 0, 0, (const uint2*)buf, out);
    hipLaunchKernelGGL(k_cal_coal4, grid, blk, 0, 0, (const uint32_t*)buf + (1u << 26), out);
    hipLaunchKernelGGL(k_cal_seg64, grid, blk, 0, 0, (const uint4*)buf, out);
    hipLaunchKernelGGL(k_cal_wstream16, grid, blk, 0, 0, (uint4*)buf);
    hipLaunchKernelGGL(k_cal_wrec12, grid, blk, 0, 0, (uint32_t*)buf);
    hipLaunchKernelGGL(k_cal_wword4, grid, blk, 0, 0, (uint32_t*)buf);
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 1;
    }
    printf("accesses per kernel: %u\n", kN);
    hipFree(buf);
    hipFree(out);
    return 0;
}
