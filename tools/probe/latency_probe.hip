// latency_probe.hip — dependent-load latency on MI355X for the engine's access
// pattern (developer measurement, not product code).  Each wavefront owns a
// region of S bytes (like a replica arena) and does K dependent rounds; in a
// round all 64 lanes load one random 64-B line each (a route-window gather)
// and the next round's addresses depend on every lane's value.  Prints ns per
// round for several region sizes and wave counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

template <int LOADS, int LINES>
__global__ __launch_bounds__(64) void chase(const uint64_t* __restrict__ buf, uint64_t words_per_wave, int rounds,
                                            int lanes, uint64_t* out) {
    const uint64_t* base = buf + (uint64_t)blockIdx.x * words_per_wave;
    const uint64_t lines = words_per_wave / 8;
    uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x + 1) + threadIdx.x * 0xBF58476D1CE4E5B9ull;
    uint64_t acc = 0;
    for (int r = 0; r < rounds; r++) {
        x ^= acc;
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        uint64_t v = 0;
        if ((int)threadIdx.x < lanes) {
            // LOADS 16-B loads from the same 64-B line, on each of LINES lines
            for (int l = 0; l < LINES; l++) {
                const uint64_t* ln = base + ((((x >> 17) + l * 0x9E3779B1ull) % lines) * 8);
                for (int k = 0; k < LOADS; k++) {
                    const uint4 q = *reinterpret_cast<const uint4*>(ln + 2 * (k & 3));
                    v += q.x ^ q.w;
                }
            }
        }
        // every lane's value feeds the next round
        uint64_t m = v;
        for (int o = 32; o >= 1; o >>= 1) m ^= __shfl_xor(m, o, 64);
        acc = m;
    }
    if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    size_t free_b, total_b;
    hipMemGetInfo(&free_b, &total_b);
    const uint64_t S = 152ull << 20;
    const int rounds = 2000;
    uint64_t* out;
    hipMalloc(&out, 4096 * 8);
    for (int waves : {256, 1536}) {
        uint64_t bytes = S * (uint64_t)waves;
        uint64_t* buf;
        if (bytes > free_b * 0.9 || hipMalloc(&buf, bytes) != hipSuccess) continue;
        hipMemset(buf, 0, bytes);
        for (int lanes : {1, 22, 64}) {
            for (int mode = 0; mode < 4; mode++) {
                hipEvent_t a, b;
                hipEventCreate(&a);
                hipEventCreate(&b);
                auto run = [&](int r) {
                    switch (mode) {
                        case 0: chase<1, 1><<<waves, 64>>>(buf, S / 8, r, lanes, out); break;
                        case 1: chase<4, 1><<<waves, 64>>>(buf, S / 8, r, lanes, out); break;
                        case 2: chase<1, 2><<<waves, 64>>>(buf, S / 8, r, lanes, out); break;
                        default: chase<4, 2><<<waves, 64>>>(buf, S / 8, r, lanes, out); break;
                    }
                };
                run(50);
                hipEventRecord(a);
                run(rounds);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                const int ld[4] = {1, 4, 1, 4}, li[4] = {1, 1, 2, 2};
                printf("waves %5d  lanes %2d  loads/line %d  lines/lane %d : %7.1f ns/round\n", waves, lanes, ld[mode],
                       li[mode], ms * 1e6 / rounds);
                fflush(stdout);
            }
        }
        hipFree(buf);
    }
    return 0;
}
