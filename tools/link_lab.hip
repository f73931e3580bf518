// link_lab.hip — what a scattered read of mapped host memory costs over
// PCIe (the zero-copy decode's h2d bytes were modelled
// as 128-byte lines; this measures the link's request granularity instead).
//
// 1M (and 4M) lanes each read `bytes` (16 .. 256, in 16-byte dwordx4
// granules, 16-byte aligned) at base + i * stride of a hipHostMalloc'd
// mapped buffer — the decode's header window loads on a socket buffer —
// and the time is compared across sizes at one stride: equal times for 16
// and 64 bytes mean the link moves (at least) 64 bytes per scattered
// request. Strides: 1,936 B (configs[2]'s mean record), 300 B (configs[1]),
// and `bytes` itself (a contiguous sweep: the link's streaming read rate).
// Also a 16-byte read at every record start whose window straddles a line
// (offset 120 within a 128-byte line): two requests or one?
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/link_lab.hip -o tools/link_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int kGran>
__global__ __launch_bounds__(256) void scatter_read(const uint8_t* base, uint64_t n, uint64_t stride, uint64_t off,
                                                    uint32_t* sink) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    uint32_t acc = 0;
    if (i < n) {
        const uint8_t* p = base + i * stride + off;
        u32x4 v[kGran];
#pragma unroll
        for (int k = 0; k < kGran; ++k) v[k] = *reinterpret_cast<const u32x4*>(p + 16 * k);
#pragma unroll
        for (int k = 0; k < kGran; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;             // (keeps the loads)
}

// kLoads dwordx4 loads per lane of which only the first `nd` granules are
// distinct: loads past them re-read the last one (the decode's round-1
// pattern, clamped to the record's last granule): do the re-reads cross
// the link again?
template <int kLoads>
__global__ __launch_bounds__(256) void clamp_read(const uint8_t* base, uint64_t n, uint64_t stride, uint32_t nd,
                                                  uint32_t* sink) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    uint32_t acc = 0;
    if (i < n) {
        const uint8_t* p = base + i * stride;
        u32x4 v[kLoads];
#pragma unroll
        for (int k = 0; k < kLoads; ++k)
            v[k] = *reinterpret_cast<const u32x4*>(p + 16 * (uint32_t(k) < nd ? k : nd - 1));
#pragma unroll
        for (int k = 0; k < kLoads; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// The same bytes read cooperatively: kGran lanes per record, lane g of a
// record loading its granule g — one instruction covers 64 / kGran records'
// contiguous 16 * kGran bytes each (does the link see fewer requests?)
template <int kGran>
__global__ __launch_bounds__(256) void coop_read(const uint8_t* base, uint64_t n, uint64_t stride, uint32_t* sink) {
    const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t i = t / kGran;
    uint32_t acc = 0;
    if (i < n) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(base + i * stride + 16 * (t % kGran));
        acc = v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const uint64_t kMax = (1ull << 30) * 9 / 4;          // 2.25 GiB of mapped host memory
    // "reg": plain pages registered with hipHostRegister (what
    // onc_host_register does to a socket buffer) instead of hipHostMalloc
    const bool reg = argc > 1 && std::string(argv[1]) == "reg";
    uint8_t* h = nullptr;
    if (reg) {
        h = static_cast<uint8_t*>(std::aligned_alloc(4096, kMax));
        if (!h) return 1;
        CK(hipHostRegister(h, kMax, hipHostRegisterMapped | hipHostRegisterPortable));
    } else {
        CK(hipHostMalloc(reinterpret_cast<void**>(&h), kMax, hipHostMallocMapped));
    }
    printf("# memory: %s\n", reg ? "aligned_alloc + hipHostRegister" : "hipHostMalloc");
    for (uint64_t k = 0; k < kMax; k += 4096) h[k] = uint8_t(k >> 12);
    uint8_t* d = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    uint32_t* sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("# link_lab: scattered reads of mapped host memory (hipHostMalloc), one dwordx4 per 16 B per lane; "
           "median of 5 after a warm-up\n");
    printf("%-10s %-8s %-6s %-6s %10s %12s %14s %14s %14s\n", "records", "stride", "bytes", "off", "us", "Mreq/s",
           "GB/s asked", "GB/s @64B/req", "GB/s @128B/req");
    struct Cfg { uint64_t n, stride, bytes, off; };
    std::vector<Cfg> cfgs;
    for (uint64_t stride : {uint64_t(1936), uint64_t(300)})
        for (uint64_t b : {16, 32, 48, 64, 128, 256}) cfgs.push_back({uint64_t(1) << 20, stride, b, 0});
    cfgs.push_back({uint64_t(1) << 20, 1936, 16, 120});   // 16 bytes straddling a 128-byte line boundary
    cfgs.push_back({uint64_t(1) << 20, 1936, 16, 56});    // ... a 64-byte boundary
    for (uint64_t b : {16, 64, 256}) cfgs.push_back({uint64_t(1) << 22, b, b, 0});     // contiguous sweeps
    for (const Cfg& c : cfgs) {
        if (c.n * c.stride + c.off + c.bytes > kMax) continue;
        std::vector<float> t;
        for (int rep = 0; rep < 6; ++rep) {
            const dim3 g(uint32_t((c.n + 255) / 256));
            CK(hipEventRecord(e0, 0));
            switch (c.bytes / 16) {
                case 1: hipLaunchKernelGGL(scatter_read<1>, g, dim3(256), 0, 0, d, c.n, c.stride, c.off, sink); break;
                case 2: hipLaunchKernelGGL(scatter_read<2>, g, dim3(256), 0, 0, d, c.n, c.stride, c.off, sink); break;
                case 3: hipLaunchKernelGGL(scatter_read<3>, g, dim3(256), 0, 0, d, c.n, c.stride, c.off, sink); break;
                case 4: hipLaunchKernelGGL(scatter_read<4>, g, dim3(256), 0, 0, d, c.n, c.stride, c.off, sink); break;
                case 8: hipLaunchKernelGGL(scatter_read<8>, g, dim3(256), 0, 0, d, c.n, c.stride, c.off, sink); break;
                default: hipLaunchKernelGGL(scatter_read<16>, g, dim3(256), 0, 0, d, c.n, c.stride, c.off, sink); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double us = t[t.size() / 2] * 1e3;
        printf("%-10lu %-8lu %-6lu %-6lu %10.1f %12.1f %14.2f %14.2f %14.2f\n", (unsigned long)c.n,
               (unsigned long)c.stride, (unsigned long)c.bytes, (unsigned long)c.off, us, c.n / us,
               c.n * c.bytes / us / 1e3, c.n * 64.0 * ((c.bytes + 63) / 64) / us / 1e3,
               c.n * 128.0 * ((c.bytes + 127) / 128) / us / 1e3);
    }
    // re-reads: 4 loads per record, 1..4 distinct granules (stride 1936)
    printf("# clamped re-reads: 4 dwordx4 loads per lane at stride 1936, `distinct` of them distinct granules\n");
    for (uint32_t nd = 1; nd <= 4; ++nd) {
        std::vector<float> t;
        const uint64_t n = uint64_t(1) << 20;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(clamp_read<4>, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, 0, d, n, uint64_t(1936),
                               nd, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("loads 4 distinct %u: %10.1f us\n", nd, t[t.size() / 2] * 1e3);
    }
    // cooperative rows against the per-lane rows above (same bytes per record)
    printf("# cooperative: kGran lanes per record, one 16-byte granule each (stride 1936 and 300)\n");
    for (uint64_t stride : {uint64_t(1936), uint64_t(300)}) {
        for (int g : {1, 2, 3, 4, 8}) {
            const uint64_t n = uint64_t(1) << 20;
            std::vector<float> t;
            for (int rep = 0; rep < 6; ++rep) {
                const dim3 grid(uint32_t((n * g + 255) / 256));
                CK(hipEventRecord(e0, 0));
                switch (g) {
                    case 1: hipLaunchKernelGGL(coop_read<1>, grid, dim3(256), 0, 0, d, n, stride, sink); break;
                    case 2: hipLaunchKernelGGL(coop_read<2>, grid, dim3(256), 0, 0, d, n, stride, sink); break;
                    case 3: hipLaunchKernelGGL(coop_read<3>, grid, dim3(256), 0, 0, d, n, stride, sink); break;
                    case 4: hipLaunchKernelGGL(coop_read<4>, grid, dim3(256), 0, 0, d, n, stride, sink); break;
                    default: hipLaunchKernelGGL(coop_read<8>, grid, dim3(256), 0, 0, d, n, stride, sink); break;
                }
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            printf("coop stride %lu bytes %d: %10.1f us\n", (unsigned long)stride, 16 * g, t[t.size() / 2] * 1e3);
        }
    }
    if (reg) {
        CK(hipHostUnregister(h));
        std::free(h);
    } else {
        CK(hipHostFree(h));
    }
    return 0;
}
