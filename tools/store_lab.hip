// store_lab.hip — cache-policy bits of streaming stores on gfx950 (dev tool).
//
// A 256 MiB copy (16 B per lane, two loads in flight) whose stores carry a
// given policy (none / nt / sc1 / nt sc1 / sc0 sc1 / nt sc0 sc1), followed by
// a read of another 320 MiB buffer: the second kernel pays for whatever the
// first left dirty in L2 / the Infinity Cache, so the pair shows the policy's
// cost to the next kernel too (enc_emit -> decode in the product step).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/store_lab.hip -o tools/store_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
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

template <int P>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
    if constexpr (P == 0) *p = v;
    else if constexpr (P == 1) __builtin_nontemporal_store(v, p);
    else if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
}

template <int P>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint64_t n16) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += 2 * stride) {
        const u32x4 a = in[i];
        const u32x4 b = i + stride < n16 ? in[i + stride] : u32x4{0, 0, 0, 0};
        st16<P>(out + i, a);
        if (i + stride < n16) st16<P>(out + i + stride, b);
    }
}

template <int P>
__global__ __launch_bounds__(256) void write_k(u32x4* __restrict__ out, uint64_t n16) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride)
        st16<P>(out + i, u32x4{uint32_t(i), 1, 2, 3});
}

__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ in, uint64_t n16, uint32_t* sink) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint32_t x = 0;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = in[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) sink[0] = x;
}

// Clean-state ceilings: before every timed kernel, a 1 GiB read (every
// dirty line written back, the Infinity Cache refilled with clean data
// that the timed kernel never touches). Read-only, NT-write-only and
// NT copy of enc_emit's configs[1] volumes (read 320 MB = 256 MB payload +
// 64 MB descriptors, write 300 MB wire).
static void clean_ceilings(const u32x4* scrub, uint64_t scrub16, uint32_t* sink) {
    const size_t rb = size_t(320) * 1000 * 1000, wb = size_t(300) * 1000 * 1000;
    void *src, *dst;
    CK(hipMalloc(&src, rb));
    CK(hipMalloc(&dst, wb));
    CK(hipMemset(src, 3, rb));
    CK(hipMemset(dst, 0, wb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[4] = {"read 320 MB", "nt write 300 MB", "plain write 300 MB", "nt copy 300 MB (read 300, write 300)"};
    std::vector<float> t[4];
    for (int rep = 0; rep < 12; ++rep) {
        for (int k = 0; k < 4; ++k) {
            hipLaunchKernelGGL(read_k, dim3(8192), dim3(256), 0, 0, scrub, scrub16, sink);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            if (k == 0) hipLaunchKernelGGL(read_k, dim3(8192), dim3(256), 0, 0, (const u32x4*)src, rb / 16, sink);
            if (k == 1) hipLaunchKernelGGL(write_k<1>, dim3(8192), dim3(256), 0, 0, (u32x4*)dst, wb / 16);
            if (k == 2) hipLaunchKernelGGL(write_k<0>, dim3(8192), dim3(256), 0, 0, (u32x4*)dst, wb / 16);
            if (k == 3) hipLaunchKernelGGL(copy_k<1>, dim3(4096), dim3(256), 0, 0, (const u32x4*)src, (u32x4*)dst, wb / 16);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 2) t[k].push_back(ms * 1000.f);
        }
    }
    printf("clean-state ceilings (1 GiB read before every kernel):\n");
    for (int k = 0; k < 4; ++k) {
        std::sort(t[k].begin(), t[k].end());
        const float m = t[k][t[k].size() / 2];
        const double bytes = k == 0 ? rb : (k == 3 ? 2.0 * wb : double(wb));
        printf("  %-38s %8.1f us  %6.2f TB/s\n", names[k], m, bytes / (m * 1e-6) / 1e12);
    }
    CK(hipFree(src));
    CK(hipFree(dst));
}

// Copy variants for the clean-state copy ceiling: a wave copies kK KiB
// blocks (lane l: bytes 16l + 1024k, all kK loads issued before the first
// store), blocks assigned by a grid-stride over the buffer; P = store policy,
// LNT = nontemporal loads.
template <int kK, int P, bool LNT>
__global__ __launch_bounds__(256) void copy_blk_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint64_t n16) {
    const uint64_t waves = uint64_t(gridDim.x) * 4;
    const int lane = threadIdx.x & 63;
    for (uint64_t b = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); b * 64 * kK < n16; b += waves) {
        const uint64_t o = b * 64 * kK + lane;
        u32x4 v[kK];
#pragma unroll
        for (int k = 0; k < kK; ++k)
            if (o + 64 * k < n16) v[k] = LNT ? __builtin_nontemporal_load(in + o + 64 * k) : in[o + 64 * k];
#pragma unroll
        for (int k = 0; k < kK; ++k)
            if (o + 64 * k < n16) st16<P>(out + o + 64 * k, v[k]);
    }
}

// Tile-structured copies (enc_emit's shape): a wave streams a contiguous
// tile of kT KiB in 1 KiB steps, kD steps of loads in flight; or (kIL) the
// 4 waves of a workgroup share a 4 x kT KiB tile, wave w taking steps
// w, w + 4, ... so that the resident waves' accesses stay compact.
template <int kT, int kD, bool kIL>
__global__ __launch_bounds__(256) void copy_tile_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint64_t n16) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t base, step;
    if (kIL) { base = uint64_t(blockIdx.x) * 4 * kT * 64 + uint64_t(w) * 64; step = 4 * 64; }
    else { base = (uint64_t(blockIdx.x) * 4 + w) * kT * 64; step = 64; }
    u32x4 v[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) {
        const uint64_t o = base + d * step + lane;
        if (o < n16) v[d] = in[o];
    }
    for (int s = 0; s < kT; s += kD) {
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            const uint64_t o = base + uint64_t(s + d) * step + lane;
            const uint64_t on = base + uint64_t(s + d + kD) * step + lane;
            const u32x4 x = v[d];
            if (s + d + kD < kT && on < n16) v[d] = in[on];
            if (s + d < kT && o < n16) __builtin_nontemporal_store(x, out + o);
        }
    }
}

// Channel-camping probe: tiles of kT KiB at a stride of kT KiB, a wave
// streaming its tile in 1 KiB steps (1 in flight); kRot: the wave starts at
// step (tile mod kT) and wraps, so waves at the same moment touch different
// offsets of their tiles.
template <int kT, bool kRot>
__global__ __launch_bounds__(256) void copy_tile_rot_k(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                       uint64_t n16) {
    const int lane = threadIdx.x & 63;
    const uint64_t tile = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const uint64_t base = tile * kT * 64;
    const int rot = kRot ? int(tile % kT) : 0;
    for (int s = 0; s < kT; ++s) {
        int j = s + rot;
        if (j >= kT) j -= kT;
        const uint64_t o = base + uint64_t(j) * 64 + lane;
        if (o < n16) __builtin_nontemporal_store(in[o], out + o);
    }
}

static void copy_variants(const u32x4* scrub, uint64_t scrub16, uint32_t* sink) {
    const size_t wb = size_t(300) * 1000 * 1000;
    void *src, *dst;
    CK(hipMalloc(&src, wb));
    CK(hipMalloc(&dst, wb));
    CK(hipMemset(src, 3, wb));
    CK(hipMemset(dst, 0, wb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V { const char* name; void (*f)(const u32x4*, u32x4*, uint64_t); int grid; };
    const V vs[] = {
        {"blk 2 KiB/wave, nt st, grid 2048", copy_blk_k<2, 1, false>, 2048},
        {"blk 4 KiB/wave, nt st, grid 2048", copy_blk_k<4, 1, false>, 2048},
        {"blk 4 KiB/wave, nt st, grid 1024", copy_blk_k<4, 1, false>, 1024},
        {"blk 8 KiB/wave, nt st, grid 1024", copy_blk_k<8, 1, false>, 1024},
        {"blk 4 KiB/wave, nt ld+st, grid 2048", copy_blk_k<4, 1, true>, 2048},
        {"blk 4 KiB/wave, sc0 sc1 nt st, g 2048", copy_blk_k<4, 5, false>, 2048},
        {"blk 4 KiB/wave, plain st, grid 2048", copy_blk_k<4, 0, false>, 2048},
        {"blk 4 KiB/wave, nt st, one pass", copy_blk_k<4, 1, false>, int((wb / 16 / 256 + 3) / 4)},
        {"blk 1 KiB/wave, nt st, one pass", copy_blk_k<1, 1, false>, int((wb / 16 / 64 + 3) / 4)},
        {"tile 16 KiB/wave, 1 step in flight", copy_tile_k<16, 1, false>, int((wb / 16 / 1024 + 3) / 4)},
        {"tile 16 KiB/wave, 2 steps in flight", copy_tile_k<16, 2, false>, int((wb / 16 / 1024 + 3) / 4)},
        {"tile 4 KiB/wave, 2 steps in flight", copy_tile_k<4, 2, false>, int((wb / 16 / 256 + 3) / 4)},
        {"tile 64 KiB/WG interleaved, 2 in flight", copy_tile_k<16, 2, true>, int((wb / 16 / 1024 + 3) / 4)},
        {"tile 16 KiB/WG interleaved, 2 in flight", copy_tile_k<4, 2, true>, int((wb / 16 / 256 + 3) / 4)},
        {"blk 2 KiB/wave, nt st, one pass", copy_blk_k<2, 1, false>, int((wb / 16 / 128 + 3) / 4)},
        {"blk 1 KiB/wave, nt st, grid 2048", copy_blk_k<1, 1, false>, 2048},
        {"blk 1 KiB/wave, nt st, grid 8192", copy_blk_k<1, 1, false>, 8192},
        {"tile 4 KiB/wave, 1 step in flight", copy_tile_k<4, 1, false>, int((wb / 16 / 256 + 3) / 4)},
        {"tile 2 KiB/wave, 1 step in flight", copy_tile_k<2, 1, false>, int((wb / 16 / 128 + 3) / 4)},
        {"tile 8 KiB/wave, 2 steps in flight", copy_tile_k<8, 2, false>, int((wb / 16 / 512 + 3) / 4)},
        {"camp: tile 16 KiB, in order", copy_tile_rot_k<16, false>, int((wb / 16 / 1024 + 3) / 4)},
        {"camp: tile 16 KiB, rotated start", copy_tile_rot_k<16, true>, int((wb / 16 / 1024 + 3) / 4)},
        {"camp: tile 18 KiB, in order", copy_tile_rot_k<18, false>, int((wb / 16 / 1152 + 3) / 4)},
        {"camp: tile 19 KiB, in order", copy_tile_rot_k<19, false>, int((wb / 16 / 1216 + 3) / 4)},
        {"camp: tile 19 KiB, rotated start", copy_tile_rot_k<19, true>, int((wb / 16 / 1216 + 3) / 4)},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    std::vector<float> t[32];
    for (int rep = 0; rep < 10; ++rep) {
        for (int k = 0; k < nv; ++k) {
            hipLaunchKernelGGL(read_k, dim3(8192), dim3(256), 0, 0, scrub, scrub16, sink);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(vs[k].f, dim3(vs[k].grid), dim3(256), 0, 0, (const u32x4*)src, (u32x4*)dst, wb / 16);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 2) t[k].push_back(ms * 1000.f);
        }
    }
    printf("clean-state copies of 300 MB (read 300 + write 300):\n");
    for (int k = 0; k < nv; ++k) {
        std::sort(t[k].begin(), t[k].end());
        const float m = t[k][t[k].size() / 2];
        printf("  %-40s %8.1f us  %6.2f TB/s\n", vs[k].name, m, 2.0 * wb / (m * 1e-6) / 1e12);
    }
    CK(hipFree(src));
    CK(hipFree(dst));
}

int main() {
    const size_t nb = size_t(256) << 20, ob = size_t(320) << 20;
    void *src, *dst, *other;
    uint32_t* sink;
    CK(hipMalloc(&src, nb));
    CK(hipMalloc(&dst, nb));
    CK(hipMalloc(&other, ob));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, nb));
    CK(hipMemset(other, 2, ob));
    const uint64_t n16 = nb / 16, o16 = ob / 16;
    const char* names[7] = {"plain", "nt", "sc1", "sc1 nt", "sc0 sc1", "sc0 sc1 nt", "sc0"};
    typedef void (*CopyF)(const u32x4*, u32x4*, uint64_t);
    typedef void (*WriteF)(u32x4*, uint64_t);
    CopyF cf[7] = {copy_k<0>, copy_k<1>, copy_k<2>, copy_k<3>, copy_k<4>, copy_k<5>, copy_k<6>};
    WriteF wf[7] = {write_k<0>, write_k<1>, write_k<2>, write_k<3>, write_k<4>, write_k<5>, write_k<6>};
    std::vector<float> t[7][4];
    hipEvent_t e[3];
    for (auto& x : e) CK(hipEventCreate(&x));
    for (int rep = 0; rep < 12; ++rep) {
        for (int p = 0; p < 7; ++p) {
            for (int mode = 0; mode < 2; ++mode) {
                CK(hipMemset(other, rep, ob));   // a third buffer's traffic in between: no carry-over
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e[0], 0));
                if (mode == 0)
                    hipLaunchKernelGGL(cf[p], dim3(4096), dim3(256), 0, 0, (const u32x4*)src, (u32x4*)dst, n16);
                else
                    hipLaunchKernelGGL(wf[p], dim3(8192), dim3(256), 0, 0, (u32x4*)dst, n16);
                CK(hipEventRecord(e[1], 0));
                hipLaunchKernelGGL(read_k, dim3(8192), dim3(256), 0, 0, (const u32x4*)other, o16, sink);
                CK(hipEventRecord(e[2], 0));
                CK(hipEventSynchronize(e[2]));
                float a, b;
                CK(hipEventElapsedTime(&a, e[0], e[1]));
                CK(hipEventElapsedTime(&b, e[1], e[2]));
                if (rep >= 2) {
                    t[p][2 * mode].push_back(a * 1000.f);
                    t[p][2 * mode + 1].push_back(b * 1000.f);
                }
            }
        }
    }
    printf("%-12s %12s %12s %12s | %12s %12s %12s\n", "store policy", "copy256", "next rd320", "sum", "write256",
           "next rd320", "sum");
    for (int p = 0; p < 7; ++p) {
        float m[4];
        for (int k = 0; k < 4; ++k) {
            std::sort(t[p][k].begin(), t[p][k].end());
            m[k] = t[p][k][t[p][k].size() / 2];
        }
        printf("%-12s %12.1f %12.1f %12.1f | %12.1f %12.1f %12.1f\n", names[p], m[0], m[1], m[0] + m[1], m[2], m[3],
               m[2] + m[3]);
    }
    void* scrub;
    const size_t sb = size_t(1) << 30;
    CK(hipMalloc(&scrub, sb));
    CK(hipMemset(scrub, 7, sb));
    clean_ceilings((const u32x4*)scrub, sb / 16, sink);
    copy_variants((const u32x4*)scrub, sb / 16, sink);
    return 0;
}
