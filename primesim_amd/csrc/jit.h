// jit.h — compile-time configuration of the engine kernel (jit.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/primeuncore.h"
#include "geometry.h"

namespace pu {

// The launch shapes of the engine compiled for one configuration: fixed
// ranges / time-sliced / replica pool / resident (f[0..3]) x queue headers in
// HBM or in LDS (f[.][0..1]; the pool runs with headers in HBM only, the
// resident kernel with headers in LDS only).
// Code objects come from the offline compiler (hipcc, at build time: jit_warm)
// or from hipRTC (in-process, on a cache miss at run time).
constexpr int kJitRtc = 0, kJitOffline = 1;
// Two code objects per configuration (jit.cpp): part 0 the throughput
// kernels (f[s][0]), part 1 the latency kernels (f[s][1]).
constexpr int kJitParts = 2;
struct JitKernels {
    hipModule_t mod[kJitParts] = {nullptr, nullptr};
    int cc[kJitParts] = {0, 0};   // kJitRtc / kJitOffline: which compiler built each part
    hipFunction_t f[4][2] = {{nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}};
    bool ok = false;
    std::string key;
};

bool jit_enabled();
// The library is about to touch HIP: from now on no compiler process is started.
void jit_note_gpu();
std::string jit_source_tag();
std::string jit_key(const Geo& g, int waves_1level, const std::string& arch, int part, int cc);
// Load (compiling on a cache miss) the kernels of configuration g; leaves
// out->ok false, after a message, when the specialisation is off or fails.
int jit_load(const Geo& g, JitKernels* out, bool verbose);
// Compile into the cache without a GPU; 1 = already cached, 0 = compiled.
int jit_warm(const Geo& g, std::string* key_out);
void jit_unload(JitKernels* k);
int jit_prof_read(unsigned long long* out, int n, int reset);
int jit_launch(const JitKernels& k, bool sliced, bool lds_headers, int nblocks, hipStream_t stream, const Geo* d_geo,
               char* arena, int replica0, const pu_req* reqs, const uint64_t* off, int32_t* delays, uint64_t* pos,
               uint64_t budget_ticks, uint32_t flags, uint32_t* sched = nullptr, int nrep = 0);
// The resident kernel (engine.hip resident_body) for replica `replica`: one
// two-wave workgroup on `stream` serving the mailbox `mbox` (device-visible
// pointer) with `stage` (cap requests of device memory) until a STOP command
// or `idle_ticks` of s_memrealtime without one.
int jit_launch_resident(const JitKernels& k, hipStream_t stream, const Geo* d_geo, char* arena, int replica,
                        pu_req* stage, void* mbox, uint64_t idle_ticks, int cap);
// One-wave workgroups of the throughput kernel of launch mode `mode` (1
// time-sliced, 2 replica pool) per CU by hipOccupancy, and its static LDS bytes.
int jit_occupancy(const JitKernels& k, int mode, int* blocks_per_cu, int* lds_bytes);

}  // namespace pu
