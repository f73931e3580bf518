// desc_lab.hip — A/B timing of descriptor-read patterns (dev tool).
//
// 1M x 64-byte records (64 MB), one status word written per record: the
// access pattern of enc_len. Variants: lane-strided record loads (1 or 2
// records per lane), wave-contiguous loads transposed through LDS, and a
// plain contiguous read (ceiling). MALL scrubbed between launches.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/desc_lab.hip -o tools/desc_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

struct Rec { uint4 q[4]; };

__device__ __forceinline__ int32_t digest(const Rec& r) {
    return int32_t(r.q[0].x ^ r.q[1].y ^ r.q[2].z ^ r.q[3].w);
}

// lane-strided: P records per lane (one per 64-record tile of the wave)
template <int P>
__global__ __launch_bounds__(1024 / P) void v_strided(const Rec* __restrict__ d, int32_t* st, uint64_t n) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t rw = uint64_t(blockIdx.x) * 1024 + uint64_t(wv) * 64 * P;
    Rec r[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const uint64_t i = rw + 64 * k + lane;
        if (i < n) r[k] = d[i];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const uint64_t i = rw + 64 * k + lane;
        if (i < n) st[i] = digest(r[k]);
    }
}

// wave-contiguous loads (1 KB per instruction), transposed through LDS
template <int P>
__global__ __launch_bounds__(1024 / P) void v_lds(const Rec* __restrict__ d, int32_t* st, uint64_t n) {
    __shared__ uint4 s[(1024 / P / 64) * 256];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint4* sw = s + wv * 256;
    const uint64_t rw = uint64_t(blockIdx.x) * 1024 + uint64_t(wv) * 64 * P;
    const uint4* src = reinterpret_cast<const uint4*>(d + rw);
    const uint64_t nq = n > rw ? min(uint64_t(64 * P), n - rw) * 4 : 0;
    uint4 v[4 * P];
#pragma unroll
    for (int k = 0; k < 4 * P; ++k) {
        const uint64_t q = 64ull * k + lane;
        if (q < nq) v[k] = src[q];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int k = 0; k < 4; ++k) sw[64 * k + lane] = v[4 * p + k];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        Rec r;
#pragma unroll
        for (int k = 0; k < 4; ++k) r.q[k] = sw[4 * lane + k];
        const uint64_t i = rw + 64 * p + lane;
        if (i < n) st[i] = digest(r);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
}

// ceiling: plain contiguous read of the same bytes, 1 status per record
__global__ __launch_bounds__(256) void v_plain(const uint4* __restrict__ d, int32_t* st, uint64_t n) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;   // quad index
    if (i < 4 * n) {
        const uint4 q = d[i];
        const uint32_t x = q.x ^ q.y ^ q.z ^ q.w;
        const uint32_t y = __shfl_xor(x, 1) ^ __shfl_xor(x, 2);
        if ((i & 3) == 0) st[i >> 2] = int32_t(x ^ y);
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000;
    Rec* d; int32_t* st;
    CK(hipMalloc(&d, sizeof(Rec) * n));
    CK(hipMalloc(&st, 4 * n));
    CK(hipMemset(d, 7, sizeof(Rec) * n));
    void* scrub; const size_t scrub_b = size_t(512) << 20;
    CK(hipMalloc(&scrub, scrub_b));
    const uint32_t g = uint32_t((n + 1023) / 1024);
    struct V { const char* name; std::function<void()> run; std::vector<float> t; };
    std::vector<V> vs = {
        {"strided 1/lane (1024 thr)", [&] { hipLaunchKernelGGL(v_strided<1>, dim3(g), dim3(1024), 0, 0, d, st, n); }, {}},
        {"strided 2/lane (512 thr)", [&] { hipLaunchKernelGGL(v_strided<2>, dim3(g), dim3(512), 0, 0, d, st, n); }, {}},
        {"strided 4/lane (256 thr)", [&] { hipLaunchKernelGGL(v_strided<4>, dim3(g), dim3(256), 0, 0, d, st, n); }, {}},
        {"lds 1/lane (1024 thr)", [&] { hipLaunchKernelGGL(v_lds<1>, dim3(g), dim3(1024), 0, 0, d, st, n); }, {}},
        {"lds 2/lane (512 thr)", [&] { hipLaunchKernelGGL(v_lds<2>, dim3(g), dim3(512), 0, 0, d, st, n); }, {}},
        {"lds 4/lane (256 thr)", [&] { hipLaunchKernelGGL(v_lds<4>, dim3(g), dim3(256), 0, 0, d, st, n); }, {}},
        {"plain contiguous", [&] { hipLaunchKernelGGL(v_plain, dim3(uint32_t((4 * n + 255) / 256)), dim3(256), 0, 0, reinterpret_cast<const uint4*>(d), st, n); }, {}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const bool cold = getenv("LAB_WARM") == nullptr;
    for (int rep = 0; rep < 25; ++rep) {
        for (auto& v : vs) {
            if (cold) CK(hipMemsetAsync(scrub, rep, scrub_b, 0));
            CK(hipEventRecord(e0, 0));
            v.run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 5) v.t.push_back(ms * 1000.f);
        }
    }
    printf("n=%llu cold=%d\n", (unsigned long long)n, int(cold));
    for (auto& v : vs) {
        std::sort(v.t.begin(), v.t.end());
        printf("%-28s median %7.1f us  min %7.1f\n", v.name, v.t[v.t.size() / 2], v.t[0]);
    }
    return 0;
}
