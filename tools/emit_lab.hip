// emit_lab.hip — A/B timing harness for encode-emit kernel variants (dev tool).
//
// Builds the configs[1] workload (1M x Call(AuthNone x2) + 256 B payload)
// on the device, runs the product pipeline (enc_len -> scan -> enc_emit) as
// the reference output, then times experimental emit variants interleaved
// in one process (MI355X guide §5.4 rule 24) and checks each variant's
// bytes against the product output.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/emit_lab.hip -o tools/emit_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../onc-rpc_amd/csrc/encode.hip"
#include "../onc-rpc_amd/csrc/scan.hip"
namespace onc {
thread_local LaunchEvents t_launch_events{nullptr, nullptr};   // the codec library defines it (codec.hip)
}

namespace onc {
struct RecEnt {   // lab-only record entry (start, payload start, end, source base)
    uint64_t start, pst, en, srcbase;
};
}  // namespace onc

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace onc;

// ---- V_copy: ideal 16-byte grid-stride copy of the output size ----------
__global__ __launch_bounds__(256) void v_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256)
        out[i] = in[i];
}

// ---- copy variants: U 16-byte loads in flight per lane, optional nontemporal
template <int U, bool NT>
__global__ __launch_bounds__(256) void v_copy_u(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + u * stride;
            if (k < n16) { if (NT) { const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in) + k); v[u] = make_uint4(t.x, t.y, t.z, t.w); } else v[u] = in[k]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + u * stride;
            if (k < n16) { if (NT) __builtin_nontemporal_store(u32x4{v[u].x, v[u].y, v[u].z, v[u].w}, reinterpret_cast<u32x4*>(out) + k); else out[k] = v[u]; }
        }
    }
}
// copy whose source is 4-aligned but not 16-aligned (single a4 dwordx4 load)
template <int U>
__global__ __launch_bounds__(256) void v_copy_a4(const uint8_t* __restrict__ in, uint4* __restrict__ out, uint64_t n16, uint32_t shift) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    const uintptr_t src = reinterpret_cast<uintptr_t>(in) + shift;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride * U) {
        u32x4_a4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + u * stride;
            if (k < n16) v[u] = gload<u32x4_a4>(src + 16 * k);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + u * stride;
            if (k < n16) out[k] = make_uint4(v[u].x, v[u].y, v[u].z, v[u].w);
        }
    }
}
__global__ __launch_bounds__(256) void v_read(const uint4* __restrict__ in, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
template <bool NT>
__global__ __launch_bounds__(256) void v_write(uint4* __restrict__ out, uint64_t n16) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256) {
        const uint4 v = make_uint4(uint32_t(i), 1, 2, 3);
        if (NT) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(out) + i); else out[i] = v;
    }
}

// ---- V_fixed: configs[1]-only structured copy (record = arithmetic) -------
// Header chunks use the same word logic from registers; measures the cost
// of the record structure without any LDS/search machinery.
__global__ __launch_bounds__(256) void v_fixed(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out,
                                               uint64_t n, uint32_t W, uint32_t H) {
    const uint64_t total = n * W;
    const uint64_t n16 = (total + 15) / 16;
    for (uint64_t c = uint64_t(blockIdx.x) * 256 + threadIdx.x; c < n16; c += uint64_t(gridDim.x) * 256) {
        const uint64_t o = c * 16;
        const uint64_t r = o / W;
        const uint64_t st = r * W, pst = st + H, en = st + W;
        uint32_t v[4];
        if (o >= pst && o + 16 <= en) {
            load16_unaligned(reinterpret_cast<uintptr_t>(payload) + r * (W - H) + (o - pst), v);
        } else {
            v[0] = v[1] = v[2] = v[3] = 0;
        }
        if (o + 16 <= total) *reinterpret_cast<uint4*>(out + o) = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// ---- V_rec<K>: record-driven copy, K lanes per record (configs[1] shape) --
template <int K>
__global__ __launch_bounds__(256) void v_rec(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out,
                                             uint64_t n, uint32_t W, uint32_t H) {
    const uint64_t lane_rec = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / K;
    const uint32_t sub = threadIdx.x % K;
    const uint64_t stride = uint64_t(gridDim.x) * 256 / K;
    for (uint64_t r = lane_rec; r < n; r += stride) {
        const uint64_t st = r * W, pst = st + H, en = st + W;
        const uint64_t A = (pst + 15) >> 4, B = en >> 4;
        const uintptr_t sb = reinterpret_cast<uintptr_t>(payload) + r * (W - H) - pst;
        for (uint64_t c = A + sub; c < B; c += K) {
            uint32_t v[4];
            load16_unaligned(sb + (c << 4), v);
            *reinterpret_cast<uint4*>(out + (c << 4)) = make_uint4(v[0], v[1], v[2], v[3]);
        }
    }
}

// ---- V_lds: product fast-pass lookups, arithmetic staging (configs[1]) ---
template <int kWaves, int U = 1>
__global__ __launch_bounds__(64 * kWaves) void v_lds(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out,
                                                     uint64_t n, uint32_t W, uint32_t H) {
    __shared__ RecEnt s_ent[kWaves][65];
    __shared__ uint8_t s_map[kWaves][512];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t tile = uint64_t(blockIdx.x) * kWaves + wv;
    const uint64_t r0 = tile * 64;
    if (r0 >= n) return;
    const int nrec = int(min(uint64_t(64), n - r0));
    RecEnt* ent = s_ent[wv];
    uint8_t* map = s_map[wv];
    const uint64_t T0 = r0 * W, T1 = (r0 + nrec) * W, G0 = T0 >> 6;
    if (lane < nrec) {
        const uint64_t r = r0 + lane, st = r * W, pst = st + H, en = st + W;
        ent[lane] = RecEnt{st, pst, en, reinterpret_cast<uintptr_t>(payload) + r * (W - H) - pst};
        const uint64_t g_hi = min((en - 1) >> 6, G0 + 511);
        for (uint64_t g = (st + 63) >> 6; g <= g_hi; ++g) map[g - G0] = uint8_t(lane);
    }
    if (lane == 0) {
        ent[nrec] = RecEnt{T1, T1, T1, 0};
        if (T0 & 63) map[0] = 0;
    }
    wave_lds_sync();
    const uint64_t c_begin = T0 >> 4, c_end = (T1 + 15) >> 4;
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(payload);
    for (uint64_t cb = c_begin + lane; cb < c_end; cb += 64 * U) {
        uintptr_t addr[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c = cb + 64 * u;
            const uint64_t o = c << 4;
            const uint64_t lo = max(o, T0);
            const uint64_t g = min((lo >> 6) - G0, uint64_t(511));
            int r = map[g];
            RecEnt e = ent[r];
            if (lo >= e.en && r + 1 < nrec) e = ent[++r];
            ok[u] = c < c_end && o >= e.pst && o + 16 <= e.en;
            addr[u] = ok[u] ? e.srcbase + o : dummy;
        }
        uint32_t v[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) load16_unaligned(addr[u], v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) *reinterpret_cast<uint4*>(out + ((cb + 64 * u) << 4)) = make_uint4(v[u][0], v[u][1], v[u][2], v[u][3]);
    }
}

// ---- V_fixed_tiled: arithmetic lookup, but each wave owns a 64-record tile
template <bool kAll>
__global__ __launch_bounds__(256) void v_fixed_tiled(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out,
                                                     uint64_t n, uint32_t W, uint32_t H, uint32_t recs_per_wave) {
    const int lane = threadIdx.x & 63;
    const uint64_t tile = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / 64;
    const uint64_t r0 = tile * recs_per_wave;
    if (r0 >= n) return;
    const uint64_t T0 = r0 * W, T1 = min(n, r0 + recs_per_wave) * W;
    for (uint64_t c = (T0 >> 4) + lane; c < (T1 + 15) >> 4; c += 64) {
        const uint64_t o = c * 16;
        const uint64_t r = o / W;
        const uint64_t st = r * W, pst = st + H, en = st + W;
        uint32_t v[4] = {0, 0, 0, 0};
        const bool fast = o >= pst && o + 16 <= en;
        if (fast) load16_unaligned(reinterpret_cast<uintptr_t>(payload) + r * (W - H) + (o - pst), v);
        if (fast || kAll) *reinterpret_cast<uint4*>(out + o) = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// ---- V_fixed_blocktiled: block of B threads owns R records, sweeps B*16 B per step
template <int B>
__global__ __launch_bounds__(B) void v_fixed_blocktiled(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out,
                                                        uint64_t n, uint32_t W, uint32_t H, uint32_t R) {
    const uint64_t r0 = uint64_t(blockIdx.x) * R;
    if (r0 >= n) return;
    const uint64_t T0 = r0 * W, T1 = min(n, r0 + R) * W;
    for (uint64_t c = (T0 >> 4) + threadIdx.x; c < (T1 + 15) >> 4; c += B) {
        const uint64_t o = c * 16;
        const uint64_t r = o / W;
        const uint64_t st = r * W, pst = st + H, en = st + W;
        if (o >= pst && o + 16 <= en) {
            uint32_t v[4];
            load16_unaligned(reinterpret_cast<uintptr_t>(payload) + r * (W - H) + (o - pst), v);
            *reinterpret_cast<uint4*>(out + o) = make_uint4(v[0], v[1], v[2], v[3]);
        }
    }
}

// ---- V_fixed_persist: persistent waves, wave-owned R-record tiles, tile
// index strided by the number of waves in the grid
__global__ __launch_bounds__(256) void v_fixed_persist(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out,
                                                       uint64_t n, uint32_t W, uint32_t H, uint32_t R) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    for (uint64_t tile = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / 64; tile * R < n; tile += nw) {
        const uint64_t r0 = tile * R;
        const uint64_t T0 = r0 * W, T1 = min(n, r0 + R) * W;
        for (uint64_t c = (T0 >> 4) + lane; c < (T1 + 15) >> 4; c += 64) {
            const uint64_t o = c * 16;
            const uint64_t r = o / W;
            const uint64_t st = r * W, pst = st + H, en = st + W;
            if (o >= pst && o + 16 <= en) {
                uint32_t v[4];
                load16_unaligned(reinterpret_cast<uintptr_t>(payload) + r * (W - H) + (o - pst), v);
                *reinterpret_cast<uint4*>(out + o) = make_uint4(v[0], v[1], v[2], v[3]);
            }
        }
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000000;
    const uint32_t P = argc > 2 ? uint32_t(strtoul(argv[2], nullptr, 10)) : 256, H = 44, W = H + P;
    std::vector<onc_msg> msgs(n);
    for (uint64_t i = 0; i < n; ++i) {
        onc_msg& m = msgs[i];
        memset(&m, 0, sizeof(m));
        m.xid = uint32_t(i);
        m.msg_type = ONC_MSG_CALL;
        m.u.call.program = 100003;
        m.u.call.program_version = 4;
        m.u.call.procedure = 1;
        m.payload_len = P;
        m.payload_off = i * P;
        m.cred.kind_len = ONC_AUTH_PACK(ONC_KIND_NONE, 0);
        m.verf.kind_len = ONC_AUTH_PACK(ONC_KIND_NONE, 0);
    }
    std::vector<uint8_t> pay(n * P + 16);
    std::mt19937_64 rng(1);
    for (auto& b : pay) b = uint8_t(rng());

    onc_msg* d_msgs;
    uint8_t *d_pay, *d_out, *d_out2, *d_auth;
    onc_unix_params* d_unix;
    uint64_t *d_off, *d_scr;
    int32_t* d_st;
    const uint64_t tiles = num_emit_tiles(n);
    CK(hipMalloc(&d_msgs, n * sizeof(onc_msg)));
    CK(hipMalloc(&d_pay, pay.size()));
    CK(hipMalloc(&d_out, n * W + 64));
    CK(hipMalloc(&d_out2, n * W + 64));
    CK(hipMalloc(&d_auth, 64));
    CK(hipMalloc(&d_unix, sizeof(onc_unix_params)));
    CK(hipMalloc(&d_off, (n + 1) * 8));
    CK(hipMalloc(&d_scr, (3 * tiles + 2 * (tiles / 4 + 1) + 16) * 8));
    CK(hipMalloc(&d_st, n * 4));
    CK(hipMemcpy(d_msgs, msgs.data(), n * sizeof(onc_msg), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pay, pay.data(), pay.size(), hipMemcpyHostToDevice));

    EncArgs a{};
    a.n = n;
    a.msgs = d_msgs;
    a.unix = d_unix;
    a.auth_arena = d_auth;
    a.payload_arena = d_pay;
    a.bounds = Bounds{1, 64, pay.size()};
    a.out = d_out;
    a.out_cap = n * W;
    a.rec_off = d_off;
    a.status = d_st;
    a.tile_sum = d_scr;
    a.block_sum = d_scr + 3 * tiles;
    a.block_base = d_scr + 3 * tiles + tiles / 4 + 1;
    CK(launch_enc_len(a, 0));
    CK(launch_scan_tiles(a.block_sum, a.block_base, num_len_blocks(n), 0, d_off + n, 0));
    CK(launch_enc_emit(a, 0));
    CK(hipDeviceSynchronize());
    // independent host reference of the configs[1] wire: 11 header words + payload
    std::vector<uint8_t> ref(n * W);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t hdr[11] = {0x80000000u | (W - 4), uint32_t(i), 0, 2, 100003, 4, 1, 0, 0, 0, 0};
        uint8_t* r = ref.data() + i * W;
        for (int k = 0; k < 11; ++k)
            for (int b = 0; b < 4; ++b) r[4 * k + b] = uint8_t(hdr[k] >> (24 - 8 * b));
        memcpy(r + H, pay.data() + i * P, P);
    }
    {
        std::vector<uint8_t> got(n * W);
        CK(hipMemcpy(got.data(), d_out, n * W, hipMemcpyDeviceToHost));
        printf("product pipeline vs host reference: %s\n", got == ref ? "bit-exact" : "MISMATCH");
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Var {
        const char* name;
        bool check;
        std::function<void()> run;
    };
    EncArgs a2 = a;
    a2.out = d_out2;
    const uint64_t n16 = (n * W + 15) / 16;
    std::vector<Var> vars = {
        {"product_len_scan_emit", true, [&] { launch_enc_len(a2, 0); launch_scan_tiles(a2.block_sum, a2.block_base, num_len_blocks(n), 0, d_off + n, 0); launch_enc_emit(a2, 0); }},
        {"product_emit_only", false, [&] { launch_enc_emit(a2, 0); }},
        {"img_u1", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<1>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u1_ntld", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<1, 1>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u1_ntst", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<1, 2>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u1_ntboth", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<1, 3>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u2_ntboth", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<2, 3>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u2_ntst", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<2, 2>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u4_ntboth", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<4, 3>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u2", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<2>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u4", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<4>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        {"img_u8", true, [&] { hipLaunchKernelGGL((enc_emit_kernel_t<8>), dim3(uint32_t((tiles + 3) / 4)), dim3(256), 0, 0, a2); }},
        
        {"copy_256MB_payload_ideal", false,
         [&] { hipLaunchKernelGGL(v_copy, dim3(2048), dim3(256), 0, 0, (const uint4*)d_pay, (uint4*)d_out2, n * P / 16); }},
        {"copy_u4_2048", false, [&] { hipLaunchKernelGGL((v_copy_u<4, false>), dim3(2048), dim3(256), 0, 0, (const uint4*)d_pay, (uint4*)d_out2, n * P / 16); }},
        {"copy_u4_nt_2048", false, [&] { hipLaunchKernelGGL((v_copy_u<4, true>), dim3(2048), dim3(256), 0, 0, (const uint4*)d_pay, (uint4*)d_out2, n * P / 16); }},
        {"copy_u1_8192", false, [&] { hipLaunchKernelGGL((v_copy_u<1, false>), dim3(8192), dim3(256), 0, 0, (const uint4*)d_pay, (uint4*)d_out2, n * P / 16); }},
        {"copy_u2_nt_4096", false, [&] { hipLaunchKernelGGL((v_copy_u<2, true>), dim3(4096), dim3(256), 0, 0, (const uint4*)d_pay, (uint4*)d_out2, n * P / 16); }},
        {"copy_a4_shift0_8192", false, [&] { hipLaunchKernelGGL((v_copy_a4<1>), dim3(8192), dim3(256), 0, 0, d_pay, (uint4*)d_out2, n * P / 16 - 1, 0u); }},
        {"copy_a4_shift4_8192", false, [&] { hipLaunchKernelGGL((v_copy_a4<1>), dim3(8192), dim3(256), 0, 0, d_pay, (uint4*)d_out2, n * P / 16 - 1, 4u); }},
        {"copy_a4_shift4_u2_4096", false, [&] { hipLaunchKernelGGL((v_copy_a4<2>), dim3(4096), dim3(256), 0, 0, d_pay, (uint4*)d_out2, n * P / 16 - 1, 4u); }},
        {"read_256MB", false, [&] { hipLaunchKernelGGL(v_read, dim3(4096), dim3(256), 0, 0, (const uint4*)d_pay, n * P / 16, (uint32_t*)d_auth); }},
        {"write_300MB", false, [&] { hipLaunchKernelGGL((v_write<false>), dim3(4096), dim3(256), 0, 0, (uint4*)d_out2, n * W / 16); }},
        {"write_300MB_nt", false, [&] { hipLaunchKernelGGL((v_write<true>), dim3(4096), dim3(256), 0, 0, (uint4*)d_out2, n * W / 16); }},
        {"fixed_structured_copy", false,
         [&] { hipLaunchKernelGGL(v_fixed, dim3(2048), dim3(256), 0, 0, d_pay, d_out2, n, W, H); }},
        {"product_len", false, [&] { launch_enc_len(a2, 0); }},
        {"product_scan", false, [&] { launch_scan_tiles(a2.block_sum, a2.block_base, num_len_blocks(n), 0, d_off + n, 0); }},
        {"lds_lookup_copy_4w", false, [&] { hipLaunchKernelGGL(v_lds<4>, dim3((tiles + 3) / 4), dim3(256), 0, 0, d_pay, d_out2, n, W, H); }},
        
        
        {"fixed_tiled_64rec_all_stores", false, [&] { hipLaunchKernelGGL(v_fixed_tiled<true>, dim3((n / 64 + 4) / 4), dim3(256), 0, 0, d_pay, d_out2, n, W, H, 64u); }},
        {"fixed_tiled_64rec", false, [&] { hipLaunchKernelGGL(v_fixed_tiled<false>, dim3((n / 64 + 4) / 4), dim3(256), 0, 0, d_pay, d_out2, n, W, H, 64u); }},
        
        
        
        
        
        
        
        
        
        
        
        
        
        
        
        
    };
    const int reps = 10, rounds = 5;
    std::vector<std::vector<float>> times(vars.size());
    for (int round = 0; round < rounds; ++round) {
        for (size_t v = 0; v < vars.size(); ++v) {
            vars[v].run();  // warm
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) vars[v].run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            times[v].push_back(ms * 1000.f / reps);
        }
    }
    for (size_t v = 0; v < vars.size(); ++v) {
        auto t = times[v];
        std::sort(t.begin(), t.end());
        bool ok = true;
        if (vars[v].check) {
            CK(hipMemset(d_out2, 0, n * W));
            vars[v].run();
            CK(hipDeviceSynchronize());
            std::vector<uint8_t> got(n * W);
            CK(hipMemcpy(got.data(), d_out2, n * W, hipMemcpyDeviceToHost));
            ok = got == ref;
        }
        printf("%-28s median %8.1f us  min %8.1f us  %s\n", vars[v].name, t[t.size() / 2], t[0],
               vars[v].check ? (ok ? "bit-exact" : "MISMATCH") : "-");
    }
    return 0;
}
