// lookback_lab.hip — cost of the placement a single-pass encode needs (dev tool).
//
// A single-pass encode (no enc_len launch) must place every 64-record tile
// inside enc_emit: claim a tile id from a counter (start order, so a wave
// only ever waits on tiles already claimed by running waves — no deadlock
// when the grid is not fully resident), plan its 64 descriptors
// (plan_record<true>, the emit's own planner), publish the tile's byte total,
// look back over the predecessors' published totals (decoupled look-back)
// for its base, publish its inclusive prefix. This lab runs exactly that
// and nothing else over a configs[1] batch, so its time is what the emit's
// tiles would pay on top of their streaming — against enc_len's 13.7 us
// (profiles/bench_r05_default.log) and the measured upper bound of the
// whole single-pass idea (tools/single_pass_bound.py). Checked against a
// host prefix sum.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lookback_lab.hip -o tools/lookback_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../onc-rpc_amd/csrc/common.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace onc;

constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62, kVal = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;     // a wave that spins this long gives up (flag), never hangs

__device__ __forceinline__ uint64_t ld_state(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_state(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// kW: predecessor states read per lane per look-back round (64 * kW per round)
template <int kW>
__global__ __launch_bounds__(256) void lookback_kernel(const onc_msg* msgs, uint64_t n, Bounds bd, uint32_t* ctr,
                                                       uint64_t* state, uint64_t* base_out, uint32_t* fail) {
    const int lane = threadIdx.x & 63;
    const uint64_t ntiles = (n + 63) / 64;
    for (;;) {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ctr, 1u);
        t = uint32_t(__builtin_amdgcn_readfirstlane(int(t)));
        if (t >= ntiles) break;
        const uint64_t r = uint64_t(t) * 64 + lane;
        MsgRegs mr = issue_msg(msgs + (r < n ? r : n - 1));
        const onc_msg d = as_msg(mr);
        const uint64_t len = r < n ? plan_record<true>(d, nullptr, bd).len : 0;
        const uint64_t agg = lane_u64(wave_incl_scan_u64(len), 63);
        if (lane == 0) st_state(state + t, kAgg | agg);
        uint64_t excl = 0;
        int64_t j = int64_t(t);             // tiles [0, j) not yet summed
        uint32_t spins = 0;
        while (j > 0) {
            uint64_t v[kW];
#pragma unroll
            for (int k = 0; k < kW; ++k) {
                const int64_t idx = j - 1 - lane - 64 * k;
                v[k] = idx >= 0 ? ld_state(state + idx) : kIncl;
            }
            // the nearest inclusive prefix (lane + 64 k order = distance), every state before it present
            bool done = false, retry = false;
            uint64_t sum = 0;
#pragma unroll
            for (int k = 0; k < kW && !done && !retry; ++k) {
                const uint64_t incl = __ballot((v[k] >> 62) == 2);
                const uint64_t empty = __ballot((v[k] >> 62) == 0);
                const int first = incl ? __builtin_ctzll(incl) : 64;
                const uint64_t upto = first == 64 ? ~0ull : ((2ull << first) - 1);   // lanes <= first
                if (empty & upto) {
                    retry = true;
                } else {
                    const uint64_t mine = uint64_t(lane) <= uint64_t(first) ? (v[k] & kVal) : 0;
                    sum += lane_u64(wave_incl_scan_u64(mine), 63);
                    if (first < 64) done = true;
                }
            }
            if (retry) {
                if (++spins > kSpinLimit) {
                    if (lane == 0) atomicOr(fail, 1u);
                    break;
                }
                continue;                  // (the sums of this round are dropped: re-read it)
            }
            excl += sum;
            if (done) break;
            j -= 64 * kW;
        }
        if (lane == 0) {
            st_state(state + t, kIncl | (excl + agg));
            base_out[t] = excl;
        }
    }
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000;
    const uint64_t ntiles = (n + 63) / 64;
    std::vector<onc_msg> m(n);
    std::vector<uint64_t> want(ntiles + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
        onc_msg& d = m[i];
        std::memset(&d, 0, sizeof(d));
        d.xid = uint32_t(i);
        d.msg_type = ONC_MSG_CALL;
        d.payload_len = 256;                   // configs[1]: AUTH_NONE x2 + 256 B: 300-byte records
        d.payload_off = 256 * i;
        want[i / 64 + 1] += 300;
    }
    for (uint64_t t = 0; t < ntiles; ++t) want[t + 1] += want[t];
    onc_msg* dm; uint32_t* ctr; uint64_t *state, *base; uint32_t* fail;
    CK(hipMalloc(&dm, n * sizeof(onc_msg)));
    CK(hipMemcpy(dm, m.data(), n * sizeof(onc_msg), hipMemcpyHostToDevice));
    CK(hipMalloc(&ctr, 4)); CK(hipMalloc(&state, 8 * ntiles)); CK(hipMalloc(&base, 8 * ntiles)); CK(hipMalloc(&fail, 4));
    CK(hipMemset(fail, 0, 4));
    const Bounds bd{0, 0, 256 * n};
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    struct Cfg { const char* name; uint32_t grid; int w; };
    const Cfg cfgs[] = {{"1024 WG x 4 waves, 256 states/round", 1024, 4}, {"1024 WG x 4 waves, 1024 states/round", 1024, 16},
                        {"4096 WG x 4 waves, 1024 states/round", 4096, 16}, {"256 WG x 4 waves, 1024 states/round", 256, 16}};
    for (const Cfg& c : cfgs) {
        std::vector<float> tk, tm;
        for (int rep = 0; rep < 12; ++rep) {
            CK(hipEventRecord(e0, 0));
            CK(hipMemsetAsync(ctr, 0, 4, 0));
            CK(hipMemsetAsync(state, 0, 8 * ntiles, 0));
            CK(hipEventRecord(e1, 0));
            if (c.w == 4) hipLaunchKernelGGL(lookback_kernel<4>, dim3(c.grid), dim3(256), 0, 0, dm, n, bd, ctr, state, base, fail);
            else hipLaunchKernelGGL(lookback_kernel<16>, dim3(c.grid), dim3(256), 0, 0, dm, n, bd, ctr, state, base, fail);
            CK(hipEventRecord(e2, 0));
            CK(hipEventSynchronize(e2));
            float a, b;
            CK(hipEventElapsedTime(&a, e0, e1));
            CK(hipEventElapsedTime(&b, e1, e2));
            if (rep >= 5) { tm.push_back(a * 1000.f); tk.push_back(b * 1000.f); }
        }
        std::vector<uint64_t> got(ntiles);
        uint32_t f = 0;
        CK(hipMemcpy(got.data(), base, 8 * ntiles, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
        bool ok = f == 0;
        for (uint64_t t = 0; t < ntiles && ok; ++t) ok = got[t] == want[t];
        std::sort(tk.begin(), tk.end());
        std::sort(tm.begin(), tm.end());
        printf("%-40s plan + look-back kernel median %6.1f us (min %6.1f); state reset (2 memsets) median %5.1f us; %s\n",
               c.name, tk[tk.size() / 2], tk[0], tm[tm.size() / 2], ok ? "bases exact" : "BASES WRONG");
    }
    return 0;
}
