// line_lab.hip — what the c2 decode's memory access alone costs.
//
// Lab (not product): the decode kernel's header-window loads on the real
// configs[2] wire without the parse — lane per record, round 1 = the chunks
// of the record's first 44 bytes, round 2 (issued after round 1 has
// arrived, as in the decode) = the rest of its header extent up to 10
// chunks — plus, optionally, the decode's 76 bytes of output per record
// (64-byte descriptor + status + 2 aux words, coalesced nontemporal stores).
// Driven by tools/line_lab.py, which times it next to the product decode.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/line_lab.hip -o tools/libline_lab.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GL __attribute__((address_space(1)))

template <bool kOut, bool kLds, int kUnix = 0>
__global__ __launch_bounds__(64) void line_kernel(const uint8_t* wire, const uint64_t* rec_off, const uint32_t* hdr,
                                                  uint64_t n, uint32_t* sink, uint8_t* out) {
    __shared__ uint32_t s_pad[kLds ? 2560 : 1];     // the decode's 10 KiB window (occupancy)
    const uint64_t i = uint64_t(blockIdx.x) * 64 + threadIdx.x;
    uint32_t acc = 0;
    if (i < n) {
        const uint64_t b = rec_off[i], L = rec_off[i + 1] - b;
        const uintptr_t base = reinterpret_cast<uintptr_t>(wire) + b;
        const uintptr_t win = base & ~uintptr_t(15);
        const uint32_t q0 = uint32_t(base - win);
        const uint32_t avail = uint32_t(min(uint64_t(10), (q0 + L + 15) >> 4));
        const uint32_t r1 = min(avail, uint32_t((q0 + min(L, uint64_t(44)) + 15) >> 4));
        u32x4 v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (j < r1) v[j] = *(const GL u32x4*)(win + 16 * j);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (j < r1) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
        const uint32_t hw = hdr[i];
        const uint32_t want = min(avail, (q0 + (hw & 0x7FFFFFFFu) + 15) >> 4);
        // round 2 depends on round 1 (the decode reads the credential length first)
        const uintptr_t win2 = win + (acc & 0x80000000u & 0u);
        u32x4 w[6];
#pragma unroll
        for (uint32_t j = 4; j < 10; ++j)
            if (j >= r1 && j < want) w[j - 4] = *(const GL u32x4*)(win2 + 16 * j);
#pragma unroll
        for (uint32_t j = 4; j < 10; ++j)
            if (j >= r1 && j < want) acc ^= w[j - 4].x ^ w[j - 4].y ^ w[j - 4].z ^ w[j - 4].w;
        if (r1 < 3 && want > r1) {      // chunk 3 of round 1 skipped but wanted
            const u32x4 x = *(const GL u32x4*)(win2 + 16 * r1);
            acc ^= x.x ^ x.w;
        }
    }
    if (kOut) {
        // 64-byte descriptor staged per workgroup: 4 KiB contiguous, 4 dwordx4 per lane
        u32x4* d = reinterpret_cast<u32x4*>(out + (uint64_t(blockIdx.x) * 64) * 64);
        const uint64_t nb = min(uint64_t(64), n - uint64_t(blockIdx.x) * 64);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = uint32_t(k * 64 + threadIdx.x);
            if (j < 4 * nb) __builtin_nontemporal_store(u32x4{acc, acc, acc, j}, d + j);
        }
        uint32_t* st = reinterpret_cast<uint32_t*>(out + n * 64);
        if (i < n) {
            __builtin_nontemporal_store(acc, st + i);
            __builtin_nontemporal_store(acc, st + n + i);
            __builtin_nontemporal_store(acc, st + 2 * n + i);
        }
    } else if (i < n) {
        sink[i] = acc;
    }
    // AUTH_UNIX slot stores. 1: the credential slot (96 B) + 32 B of the
    // verifier slot at 192 * i (the ABI's slot 2i), plain stores; 2: the same,
    // nontemporal; 3: compacted — the wave's AUTH_UNIX records take
    // consecutive 96-byte slots from the start of its 64 slot pairs.
    if (kUnix) {
        const bool u = i < n && (hdr[min(i, n - 1)] >> 31);
        const uint64_t m = __ballot(u);
        if (u) {
            if (kUnix == 3) {
                const uint32_t k = __popcll(m & ((1ull << threadIdx.x) - 1));
                u32x4* d = reinterpret_cast<u32x4*>(out + n * 76 + 192 * (uint64_t(blockIdx.x) * 64) + 96 * k);
#pragma unroll
                for (int q = 0; q < 6; ++q) d[q] = u32x4{acc, acc, uint32_t(q), acc};
            } else {
                u32x4* d = reinterpret_cast<u32x4*>(out + n * 76 + 192 * i);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    if (kUnix == 2) __builtin_nontemporal_store(u32x4{acc, acc, uint32_t(q), acc}, d + q);
                    else d[q] = u32x4{acc, acc, uint32_t(q), acc};
                }
            }
        }
    }
    if (kLds) {
        s_pad[threadIdx.x * 40] = acc;
        __syncthreads();
        if (s_pad[(threadIdx.x ^ 1) * 40] == 0x12345678u && i < n) sink[i] = 1;
    }
}

extern "C" int line_lab_run(const uint8_t* wire, const uint64_t* rec_off, const uint32_t* hdr, uint64_t n,
                            uint32_t* sink, uint8_t* out, int with_out, void* stream) {
    const dim3 g(uint32_t((n + 63) / 64));
    hipStream_t s = (hipStream_t)stream;
    switch (with_out) {       // bit 0: output stores, bit 1: 10 KiB LDS per workgroup, 4-6: + AUTH_UNIX slots (kUnix 1-3)
        case 0: hipLaunchKernelGGL((line_kernel<false, false>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
        case 1: hipLaunchKernelGGL((line_kernel<true, false>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
        case 2: hipLaunchKernelGGL((line_kernel<false, true>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
        case 3: hipLaunchKernelGGL((line_kernel<true, true>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
        case 4: hipLaunchKernelGGL((line_kernel<true, true, 1>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
        case 5: hipLaunchKernelGGL((line_kernel<true, true, 2>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
        default: hipLaunchKernelGGL((line_kernel<true, true, 3>), g, dim3(64), 0, s, wire, rec_off, hdr, n, sink, out); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
