// handoff.hip — one dependent hand-off between two waves on different CUs
// (developer measurement for DESIGN.md §5, not product code).
//
// The question it answers: sharding ONE simulation by home tile (north star;
// SURVEY §8e) turns every band change of a request's route into a dependent
// hand-off from one worker to another (9.3 per C4 access, relax_proto).  Two
// waves ping-pong a token: wave A publishes k, wave B waits for k and publishes
// k back, A waits for it; one-way hand-off = round trip / 2.  Variants:
//   * placement: same XCD (blocks 0 and 8 under round-robin dispatch) or
//     different XCDs (blocks 0 and 1);
//   * memory: coarse-grained device memory (hipMalloc), fine-grained device
//     memory, fine-grained host memory (the nearest proxy this 1-GPU box has
//     for a peer GPU's memory reached over a fabric link);
//   * payload: the token alone, or 256 B / 4 KB written before the token
//     (lane-parallel 16-B stores, then the token; the reader loads it after).
// Every access is a vector-memory instruction with the sc0 sc1 (system
// coherence) bits; nothing goes through the scalar data cache.  Every spin is
// bounded (a stuck partner sets an error word and the wave exits), so the
// grid always drains.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define SPIN_MAX (1u << 22)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st16_sys(v4u* p, v4u v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ v4u ld16_sys(const v4u* p) {
    v4u v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// flags: [0] A->B token, [32] B->A token (separate 128-B lines), payload at
// word 64 (A->B) and 64 + 1024 (B->A).  out[0] = s_memrealtime ticks for
// `iters` round trips, measured by A.
__global__ __launch_bounds__(64) void pingpong(uint32_t* flags, int iters, int a_blk, int b_blk, int payload_bytes,
                                               uint64_t* out, uint32_t* err) {
    const int me = blockIdx.x == (unsigned)a_blk ? 0 : blockIdx.x == (unsigned)b_blk ? 1 : -1;
    if (me < 0) return;
    const int ln = threadIdx.x;
    uint32_t* mine = flags + (me == 0 ? 0 : 32);
    uint32_t* theirs = flags + (me == 0 ? 32 : 0);
    v4u* pay_out = reinterpret_cast<v4u*>(flags + 64 + (me == 0 ? 0 : 1024));
    const v4u* pay_in = reinterpret_cast<const v4u*>(flags + 64 + (me == 0 ? 1024 : 0));
    const int nvec = payload_bytes / 16;
    uint32_t sink = 0;
    uint64_t t0 = 0;
    if (me == 0) t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 1; k <= iters; k++) {
        if (me == 1) {   // B waits first
            uint32_t s = 0;
            while (ld_sys(theirs) != (uint32_t)k) {
                if (++s > SPIN_MAX) { if (ln == 0) atomicOr(err, 2u); return; }
            }
            for (int v = ln; v < nvec; v += 64) { v4u x = ld16_sys(pay_in + v); sink += x.x; }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        for (int v = ln; v < nvec; v += 64) st16_sys(pay_out + v, v4u{(unsigned)k, (unsigned)k, (unsigned)k, (unsigned)k});
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ln == 0) st_sys(mine, (uint32_t)k);
        if (me == 0) {
            uint32_t s = 0;
            while (ld_sys(theirs) != (uint32_t)k) {
                if (++s > SPIN_MAX) { if (ln == 0) atomicOr(err, 1u); return; }
            }
            for (int v = ln; v < nvec; v += 64) { v4u x = ld16_sys(pay_in + v); sink += x.x; }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    if (me == 0 && ln == 0) {
        out[0] = __builtin_amdgcn_s_memrealtime() - t0;
        out[1] = sink;
    }
}

int main() {
    const int iters = 20000;
    uint64_t* out;
    uint32_t* err;
    if (hipMalloc(&out, 64) != hipSuccess || hipMalloc(&err, 4) != hipSuccess) return 1;
    const char* mem_names[3] = {"device coarse-grained (hipMalloc)", "device fine-grained",
                                "host fine-grained (hipHostMalloc coherent)"};
    printf("{\"iters\": %d, \"unit\": \"ns one-way (round trip / 2)\", \"results\": [\n", iters);
    bool first = true;
    for (int mem = 0; mem < 3; mem++) {
        uint32_t* flags = nullptr;
        const size_t bytes = 64 * 1024;
        hipError_t e;
        if (mem == 0) e = hipMalloc(&flags, bytes);
        else if (mem == 1) e = hipExtMallocWithFlags((void**)&flags, bytes, hipDeviceMallocFinegrained);
        else e = hipHostMalloc((void**)&flags, bytes, hipHostMallocCoherent);
        if (e != hipSuccess) {
            fprintf(stderr, "alloc %s failed: %s\n", mem_names[mem], hipGetErrorString(e));
            continue;
        }
        for (int place = 0; place < 2; place++) {
            const int a = 0, b = place == 0 ? 8 : 1;   // round-robin: block i on XCD i % 8
            for (int payload : {0, 256, 4096}) {
                double best = 1e30;
                for (int rep = 0; rep < 3; rep++) {
                    (void)hipMemset(flags, 0, bytes);
                    (void)hipMemset(err, 0, 4);
                    (void)hipDeviceSynchronize();
                    hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), 0, 0, flags, iters, a, b, payload, out, err);
                    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 2; }
                    uint64_t h[2];
                    uint32_t he;
                    (void)hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
                    (void)hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
                    if (he) { fprintf(stderr, "spin limit hit (%u)\n", he); return 3; }
                    const double ns = (double)h[0] * 10.0 / iters / 2.0;   // s_memrealtime: 100 MHz
                    best = ns < best ? ns : best;
                }
                printf("%s {\"memory\": \"%s\", \"placement\": \"%s\", \"payload_bytes\": %d, \"ns\": %.1f}",
                       first ? " " : ",\n ", mem_names[mem], place == 0 ? "same XCD" : "different XCDs", payload, best);
                first = false;
                fflush(stdout);
            }
        }
        if (mem == 2) (void)hipHostFree(flags);
        else (void)hipFree(flags);
    }
    printf("\n]}\n");
    return 0;
}
