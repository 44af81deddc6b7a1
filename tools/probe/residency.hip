// residency.hip — how many one-wave workgroups of a given resource shape are
// resident on one CU at once (developer measurement for DESIGN.md §7, not
// product code).
//
// The question it answers: round 4's six-waves-per-SIMD variant of the
// headline kernel (80 VGPRs, 7,152 B of LDS, 76 B of scratch per lane) ran at
// exactly half the rate with a grid of hipOccupancy's 22 blocks per CU; the
// five-wave kernel (96 VGPRs) and a six-wave kernel with less LDS did not.  A
// time-sliced launch whose grid exceeds what the device keeps resident takes
// two slices, so any overstatement halves the rate.  Each probe kernel has a
// chosen shape: VGPRs forced by a clobber of v(N-1), static LDS of the given
// size (touched), scratch through a dynamically indexed private array.  Every
// wave records its start (s_memrealtime), its hardware slot (HW_ID, XCC_ID)
// and spins a fixed time; the host counts the waves resident at once, the
// waves per CU, and the waves that started only after others had finished.
// Every spin is bounded by the clock, so the grid always drains.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

struct Rec {
    uint64_t t0, t1;
    uint32_t hw, xcc;
};

template <int V>
__device__ __forceinline__ void clobber_vgprs() {
    if constexpr (V == 64) asm volatile("" ::: "v63");
    else if constexpr (V == 80) asm volatile("" ::: "v79");
    else if constexpr (V == 96) asm volatile("" ::: "v95");
    else if constexpr (V == 128) asm volatile("" ::: "v127");
}

template <int LDS, int VG, int SCR, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void probe(Rec* out, uint64_t spin,
                                                                                       int idx) {
    __shared__ uint32_t lds[LDS > 0 ? LDS / 4 : 1];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    clobber_vgprs<VG>();
    uint32_t acc = threadIdx.x;
    if constexpr (LDS > 0) {
        for (int i = threadIdx.x; i < LDS / 4; i += 64) lds[i] = (uint32_t)i;
        __syncthreads();
        acc += lds[(threadIdx.x * 7 + idx) % (LDS / 4)];
    }
    if constexpr (SCR > 0) {
        volatile uint32_t priv[SCR];
        for (int i = 0; i < SCR; i++) priv[i] = acc + (uint32_t)i;
        acc += priv[(idx + threadIdx.x) % SCR];
    }
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(10);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        Rec r;
        r.t0 = t0;
        r.t1 = t1 + (acc == 0xFFFFFFFFu ? 1 : 0);
        r.hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_REG_HW_ID
        r.xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
        out[blockIdx.x] = r;
    }
}

template <int LDS, int VG, int SCR, int WPE>
static void run(const char* name, int cus, Rec* d, std::vector<Rec>& h, bool first) {
    auto k = probe<LDS, VG, SCR, WPE>;
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, 64, 0);
    hipFuncAttributes fa{};
    hipFuncGetAttributes(&fa, (const void*)k);
    const int grid = occ * cus;
    const uint64_t spin = 3000000;   // 30 ms at 100 MHz
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, d, spin, 1);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("%s{\"probe\": \"%s\", \"error\": \"launch failed\"}\n", first ? "" : ",", name);
        return;
    }
    hipMemcpy(h.data(), d, sizeof(Rec) * grid, hipMemcpyDeviceToHost);
    uint64_t tmin = UINT64_MAX;
    for (int i = 0; i < grid; i++) tmin = std::min(tmin, h[i].t0);
    // waves resident at once: sweep over start/end events
    std::vector<std::pair<uint64_t, int>> ev;
    int late = 0;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, int> first_wave_cu;
    for (int i = 0; i < grid; i++) {
        ev.push_back({h[i].t0, +1});
        ev.push_back({h[i].t1, -1});
        if (h[i].t0 > tmin + spin / 2) late++;
        else {
            const uint32_t hw = h[i].hw;
            // cu_id [11:8], sh_id [12], se_id [15:13] (HW_ID), xcc_id [3:0]
            first_wave_cu[{h[i].xcc & 15u, (hw >> 13) & 7u, (hw >> 12) & 1u, (hw >> 8) & 15u}]++;
        }
    }
    std::sort(ev.begin(), ev.end(), [](auto a, auto b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
    int cur = 0, mx = 0;
    for (auto& e : ev) {
        cur += e.second;
        mx = std::max(mx, cur);
    }
    int cu_min = 1 << 30, cu_max = 0;
    for (auto& kv : first_wave_cu) {
        cu_min = std::min(cu_min, kv.second);
        cu_max = std::max(cu_max, kv.second);
    }
    std::printf("%s{\"probe\": \"%s\", \"lds_bytes\": %d, \"vgprs\": %d, \"scratch_words\": %d, \"waves_per_eu\": %d, "
                "\"kernel_lds\": %zu, \"kernel_private\": %zu, \"occupancy_api_per_cu\": %d, \"grid\": %d, "
                "\"max_resident\": %d, \"late_starters\": %d, \"cus_seen\": %zu, \"first_slice_per_cu_min\": %d, "
                "\"first_slice_per_cu_max\": %d}\n",
                first ? "" : ",", name, LDS, VG, SCR, WPE, (size_t)fa.sharedSizeBytes, (size_t)fa.localSizeBytes, occ,
                grid, mx, late, first_wave_cu.size(), cu_min, cu_max);
    std::fflush(stdout);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    Rec* d = nullptr;
    const int maxgrid = 32 * cus;
    if (hipMalloc(&d, sizeof(Rec) * maxgrid) != hipSuccess) return 1;
    std::vector<Rec> h(maxgrid);
    std::printf("{\"cus\": %d, \"probes\": [\n", cus);
    // the round-4 kernels' shapes
    run<7152, 96, 5, 5>("five_waves_r4 (96 VGPR, 7152 B LDS, 20 B scratch)", cus, d, h, true);
    run<7152, 80, 19, 6>("six_waves_r4 (80 VGPR, 7152 B LDS, 76 B scratch)", cus, d, h, false);
    run<7152, 80, 0, 6>("six_waves_no_scratch", cus, d, h, false);
    run<0, 80, 19, 6>("six_waves_no_lds", cus, d, h, false);
    run<5104, 80, 19, 6>("six_waves_two_rings (5104 B LDS)", cus, d, h, false);
    run<7472, 96, 8, 5>("five_waves_r5 (96 VGPR, 7472 B LDS, 32 B scratch)", cus, d, h, false);
    // LDS size sweep at 64 VGPRs (no VGPR limit below 8 waves/SIMD)
    run<6144, 64, 0, 8>("lds_6144", cus, d, h, false);
    run<6656, 64, 0, 8>("lds_6656", cus, d, h, false);
    run<7168, 64, 0, 8>("lds_7168", cus, d, h, false);
    run<7296, 64, 0, 8>("lds_7296", cus, d, h, false);
    run<7680, 64, 0, 8>("lds_7680", cus, d, h, false);
    run<8192, 64, 0, 8>("lds_8192", cus, d, h, false);
    run<10240, 64, 0, 8>("lds_10240", cus, d, h, false);
    run<16384, 64, 0, 8>("lds_16384", cus, d, h, false);
    run<32768, 64, 0, 8>("lds_32768", cus, d, h, false);
    run<65536, 64, 0, 8>("lds_65536", cus, d, h, false);
    std::printf("]}\n");
    hipFree(d);
    return 0;
}
