// frame_lab.hip — the framer's guess and chase kernels (frame.hip) timed on
// a configs[2]-like stream (1M Call records, AUTH_NONE, payload U[64, 4096]
// random bytes) at a given chunk size. Dev tool.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I onc-rpc_amd/csrc tools/frame_lab.hip -o tools/frame_lab
#include "../onc-rpc_amd/csrc/frame.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

namespace onc {
thread_local LaunchEvents t_launch_events{nullptr, nullptr};   // defined by codec.hip in the library
}

static uint64_t sm(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void put32(std::vector<uint8_t>& b, uint64_t o, uint32_t v) {
    b[o] = v >> 24; b[o + 1] = v >> 16; b[o + 2] = v >> 8; b[o + 3] = v;
}

int main(int argc, char** argv) {
    const uint64_t n = 1000000;
    const uint64_t chunk = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    uint64_t seed = 2;
    std::vector<uint32_t> plen(n);
    uint64_t len = 0;
    for (uint64_t i = 0; i < n; ++i) { plen[i] = 64 + sm(seed) % 4033; len += 44 + plen[i]; }
    std::vector<uint8_t> w(len + 64);
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t L = 44 + plen[i];
        put32(w, o, 0x80000000u | (L - 4)); put32(w, o + 4, uint32_t(sm(seed)));
        put32(w, o + 8, 0); put32(w, o + 12, 2); put32(w, o + 16, 100003); put32(w, o + 20, 4); put32(w, o + 24, 1);
        put32(w, o + 28, 0); put32(w, o + 32, 0); put32(w, o + 36, 0); put32(w, o + 40, 0);
        for (uint32_t k = 0; k < plen[i]; k += 8) {
            const uint64_t r = sm(seed);
            for (uint32_t b = 0; b < 8 && k + b < plen[i]; ++b) w[o + 44 + k + b] = uint8_t(r >> (8 * b));
        }
        o += L;
    }
    const uint64_t P = (len + chunk - 1) / chunk;
    uint8_t* dw;
    CK(hipMalloc(&dw, len + 64));
    CK(hipMemcpy(dw, w.data(), len + 64, hipMemcpyHostToDevice));
    onc::FrameArgs a{};
    a.wire = dw; a.len = len; a.chunk = chunk; a.nchunks = P; a.max_records = n + 1;
    auto al = [](size_t b) { void* p; CK(hipMalloc(&p, b)); CK(hipMemset(p, 0, b)); return p; };
    a.rec_off = (uint64_t*)al(8 * (n + 2));
    a.starts = (uint64_t*)al(8 * 64 * P);
    a.result = (uint64_t*)al(64);
    a.g = (uint64_t*)al(8 * P); a.x = (uint64_t*)al(8 * P); a.cnt = (uint32_t*)al(4 * P); a.st = (int32_t*)al(4 * P);
    a.aux = (uint32_t*)al(8 * P); a.fail = (uint8_t*)al(P); a.stop = (uint8_t*)al(P);
    a.fail2 = (uint8_t*)al(P / 256 + 2); a.stop2 = (uint8_t*)al(P / 256 + 2);
    a.fail3 = (uint8_t*)al(P / 65536 + 2); a.stop3 = (uint8_t*)al(P / 65536 + 2);
    a.cnt_eff = (uint32_t*)al(4 * P); a.cnt_base = (uint64_t*)al(8 * P);
    a.first_fail = (uint64_t*)al(8); a.first_stop = (uint64_t*)al(8);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto f) {
        std::vector<float> v;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(e0, 0)); f(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r) v.push_back(ms * 1000);
        }
        std::sort(v.begin(), v.end());
        printf("%-28s %9.1f us\n", name, v[v.size() / 2]);
    };
    printf("stream %.1f MB, %lu chunks of %lu B\n", len / 1e6, (unsigned long)P, (unsigned long)chunk);
    timeit("frame_guess (wave/chunk)", [&] { onc::launch_frame_guess(a, 0); });
    timeit("frame_chunks (lane/chunk)", [&] { onc::launch_frame_chunks(a, 0); });
    return 0;
}
