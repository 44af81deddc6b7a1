// rcp_probe.hip — RESEARCH PROBE (not product): how accurate is gfx950's
// v_rcp_f64, and does a correctly rounded f64 division still come out with ONE
// Newton step instead of the engine's two (engine.hip rcp_nr / div_nr, which
// mirror hipcc's own lowering)?  Every thread draws random positive normal
// operands (wide exponent range, plus integers and the M/G/1 operand shapes)
// and compares, bit for bit, against the compiler's IEEE division a / b:
//   one-step  y = rcp(b); y = fma(y, fma(-b, y, 1), y);          q = a*y; q += r*y
//   two-step  the engine's (one more step before the residual correction)
// and records the largest ulp distance of the raw v_rcp_f64 from 1.0 / b.
// Output: one JSON line.  usage: rcp_probe [samples_per_thread]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint64_t mix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// a positive normal double: kind 0 random mantissa and exponent in [2^-64, 2^64),
// kind 1 an integer below 2^53, kind 2 a mantissa near 1 (cancellation shapes)
__device__ __forceinline__ double draw(uint64_t& s, int kind) {
    const uint64_t r = mix(s);
    if (kind == 1) return (double)((r >> 11) >> (r & 63 ? (r & 63) % 53 : 0)) + 1.0;
    if (kind == 2) return 1.0 + (double)(r >> 12) * 0x1p-52 * 0x1p-20;
    const uint64_t e = 1023 - 64 + (mix(s) % 128);
    return __longlong_as_double((long long)((e << 52) | (r & ((1ull << 52) - 1))));
}
__device__ __forceinline__ double div1(double a, double b) {
    double y = __builtin_amdgcn_rcp(b);
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-b, q, a), y, q);
}
__device__ __forceinline__ double div2(double a, double b) {
    double y = __builtin_amdgcn_rcp(b);
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-b, q, a), y, q);
}

__global__ void probe(uint64_t seed, int per, unsigned long long* out) {
    uint64_t s = seed ^ ((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) << 20);
    unsigned long long bad1 = 0, bad2 = 0, n = 0, rcp_max = 0, rcp_gt1 = 0;
    for (int i = 0; i < per; i++) {
        const int ka = (int)(mix(s) % 3), kb = (int)(mix(s) % 3);
        const double a = draw(s, ka), b = draw(s, kb);
        const double ref = a / b;
        bad1 += div1(a, b) != ref;
        bad2 += div2(a, b) != ref;
        const double y0 = __builtin_amdgcn_rcp(b), yr = 1.0 / b;
        const long long d = __double_as_longlong(y0) - __double_as_longlong(yr);
        const unsigned long long u = (unsigned long long)(d < 0 ? -d : d);
        rcp_max = u > rcp_max ? u : rcp_max;
        rcp_gt1 += u > 1;
        n++;
    }
    atomicAdd(&out[0], n);
    atomicAdd(&out[1], bad1);
    atomicAdd(&out[2], bad2);
    atomicMax(&out[3], rcp_max);
    atomicAdd(&out[4], rcp_gt1);
}

int main(int argc, char** argv) {
    const int per = argc > 1 ? std::atoi(argv[1]) : 4096;
    unsigned long long* d;
    if (hipMalloc(&d, 5 * 8) != hipSuccess) return 2;
    if (hipMemset(d, 0, 5 * 8) != hipSuccess) return 2;
    const int blocks = 256 * 16, threads = 256;
    probe<<<blocks, threads>>>(0x1234567ull, per, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long h[5];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("{\"samples\": %llu, \"one_step_mismatches\": %llu, \"two_step_mismatches\": %llu, "
                "\"rcp_max_ulp\": %llu, \"rcp_over_1ulp\": %llu}\n", h[0], h[1], h[2], h[3], h[4]);
    return 0;
}
