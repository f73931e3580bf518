// glds_probe.hip — does global_load_lds_dwordx4 accept 4-byte-aligned (not
// 16-byte-aligned) global addresses on gfx950, and does it return the same
// 16 bytes as global_load_dwordx4? (dev tool, one small kernel)
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/glds_probe.hip -o tools/glds_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ __forceinline__ void glds16(const void* g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}

__global__ __launch_bounds__(64) void probe(const uint8_t* src, uint4* out_dma, uint4* out_reg, uint32_t shift) {
    __shared__ uint4 ring[64];
    const int lane = threadIdx.x;
    const uint8_t* g = src + 16 * lane + shift;
    const uint32_t lds = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&ring[0]));
    glds16(g, lds);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out_dma[lane] = ring[lane];
    typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4_a4 v = *reinterpret_cast<const u32x4_a4*>(g);
    out_reg[lane] = make_uint4(v.x, v.y, v.z, v.w);
}

int main() {
    std::vector<uint8_t> h(2048);
    for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t(i * 7 + 3);
    uint8_t* d;
    uint4 *a, *b;
    hipMalloc(&d, h.size());
    hipMalloc(&a, 64 * 16);
    hipMalloc(&b, 64 * 16);
    hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
    int bad = 0;
    for (uint32_t shift : {0u, 4u, 8u, 12u}) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, a, b, shift);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("shift %u: launch failed\n", shift);
            return 1;
        }
        std::vector<uint4> ha(64), hb(64);
        hipMemcpy(ha.data(), a, 64 * 16, hipMemcpyDeviceToHost);
        hipMemcpy(hb.data(), b, 64 * 16, hipMemcpyDeviceToHost);
        int diff = 0;
        for (int l = 0; l < 64; ++l)
            diff += ha[l].x != hb[l].x || ha[l].y != hb[l].y || ha[l].z != hb[l].z || ha[l].w != hb[l].w;
        printf("shift %u: %d of 64 lanes differ (dma %08x reg %08x)\n", shift, diff, ha[1].x, hb[1].x);
        bad += diff;
    }
    printf(bad ? "MISMATCH\n" : "OK\n");
    return bad != 0;
}
