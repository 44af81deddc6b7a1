// jit.cpp — compile-time configuration of the engine kernel.
//
// A PriME configuration (the reference's XmlSys: cache geometries, mesh,
// latencies) is fixed for a whole simulation, so the engine kernel is compiled
// once per configuration with every geometry value as a constant: the
// configuration's Geo is written out as C++ (geo_emit.h), the engine's own
// sources (embedded in this library at build time, tools/embed_src.py) are
// compiled against it for gfx950, and the code object is loaded with
// hipModuleLoadData.  Two compilers: at build time (jit_warm, a process that
// has put nothing on the GPU) the ROCm driver hipcc in a child process; on a
// cache miss at run time hipRTC in-process.  The same source and options give
// different code: at C4 hipcc's throughput kernel needs 76 VGPRs and spills
// none where hipRTC's needs 80 and spills 11, +4.7% on the headline, same box
// (profiles/r5m_ab_ens.txt); so the cache prefers hipcc's object.  Constant
// geometry removes the kernel's scalar loads of its configuration and the
// scalar address arithmetic around them, the largest part of the lone wave's
// issue and wait time.
//
// Code objects are cached on disk as <source tag>-<hash of (sources, geometry,
// target arch, options)>.hsaco: PRIMEUNCORE_JIT_CACHE, else jit_cache/ next to
// libprimeuncore.so (in-tree, so a cache warmed by __graft_entry__.build()
// travels with the library; tools/jit_warm.py prunes code objects whose source
// tag no library in the tree carries).  A cached code object the device
// refuses is deleted and compiled again once.  PRIMEUNCORE_JIT=0 turns the
// specialisation off: the library's ahead-of-time kernels (the same engine
// source compiled for a runtime Geo) run instead, as they do when a compile or
// a load fails (with a message).  hipRTC itself is a link-time dependency of
// the library (-lhiprtc), not an optional one.
#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <utime.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include "common.h"
#include "geo_emit.h"
#include "jit.h"

extern const int pu_jit_nsrc;
extern const char* const pu_jit_src_name[];
extern const char* const pu_jit_src_text[];
extern char** environ;

namespace pu {
namespace {

// hipRTC compiles device code only and ships no C headers: the two the
// sources include get minimal stand-ins built on the compiler's own macros.
const char* kStdint =
    "#pragma once\n"
    "typedef __INT8_TYPE__ int8_t; typedef __UINT8_TYPE__ uint8_t;\n"
    "typedef __INT16_TYPE__ int16_t; typedef __UINT16_TYPE__ uint16_t;\n"
    "typedef __INT32_TYPE__ int32_t; typedef __UINT32_TYPE__ uint32_t;\n"
    "typedef __INT64_TYPE__ int64_t; typedef __UINT64_TYPE__ uint64_t;\n"
    "typedef __INTPTR_TYPE__ intptr_t; typedef __UINTPTR_TYPE__ uintptr_t;\n"
    "#define INT64_MAX __INT64_MAX__\n#define UINT64_MAX __UINT64_MAX__\n"
    "#define INT32_MAX __INT32_MAX__\n#define UINT32_MAX __UINT32_MAX__\n";
const char* kStddef = "#pragma once\n";

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

std::string lib_dir() {
    Dl_info info;
    if (dladdr((void*)&fnv1a, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t k = p.rfind('/');
        if (k != std::string::npos) return p.substr(0, k);
    }
    return ".";
}

std::string cache_dir() {
    if (const char* e = std::getenv("PRIMEUNCORE_JIT_CACHE"); e && *e) return e;
    return lib_dir() + "/jit_cache";
}

bool read_file(const std::string& path, std::vector<char>* out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return !out->empty();
}

void write_file_atomic(const std::string& path, const std::vector<char>& data) {
    std::string tmp = path + ".tmp." + std::to_string(::getpid());
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return;
        f.write(data.data(), (std::streamsize)data.size());
        if (!f) {
            std::remove(tmp.c_str());
            return;
        }
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

// Part 0 (the throughput kernels) of a one-level configuration is compiled
// without machine LICM: hoisted loop invariants (constants, address pairs)
// were held in SGPRs across the whole request loop and spilled (192 spill
// slots); rematerialised at their uses the kernel needs 76 VGPRs instead of 96
// and fits 6 waves per SIMD with no spill (72 and 7 waves since; engine.hip
// PU_WAVES_1LEVEL).  6 waves + 2 staged rings + this: +4.0% on the C4
// headline (profiles/r5j_ab_ens.txt, r5k_ab_ens.txt); the same flag at 5
// waves lost 1.2%, and the latency kernels lost 1.5% open / 2% closed loop
// with it (r5i_ab_nolicm.txt), so part 1 keeps the default.
std::vector<std::string> options(const std::string& arch, int waves_1level, int part, bool one_level, int cc) {
    // max-occupancy: at C4 the throughput kernel spills 2 VGPRs instead of 4
    // and ran ahead of max-ILP in each of three interleaved rounds (233.0 /
    // 230.0 / 232.7 vs 215.9 / 226.9 / 231.4 M/s), one simulation alone level
    // (profiles/r3q_ab_occ*.txt); the ahead-of-time kernels keep max-ILP.
    // -Werror=missing-field-initializers: a Geo field the emitter (geo_emit.h)
    // forgets would otherwise silently be 0 in the compiled configuration.
    std::vector<std::string> o = {"--offload-arch=" + arch, "-O3", "-std=c++20", "-ffp-contract=off", "-fwrapv",
                                  "-mllvm", "-amdgpu-sched-strategy=max-occupancy",
                                  "-DPU_JIT_GEO=\"pu_jit_geo.h\"", "-Wno-c99-designator",
                                  "-Werror=missing-field-initializers"};
    if (waves_1level > 0) o.push_back("-DPU_WAVES_1LEVEL=" + std::to_string(waves_1level));
    o.push_back("-DPU_JIT_PART=" + std::to_string(part));
    if (cc == kJitOffline)   // the ROCm compiler driver: device code only, one code object, headers written flat
        for (const char* x : {"-DPU_JIT_OFFLINE", "--cuda-device-only", "--no-gpu-bundle-output",
                              "-Wno-unused-command-line-argument"})
            o.push_back(x);
    if (part == 0 && one_level) {
        o.push_back("-mllvm");
        o.push_back("-disable-machine-licm");
    }
    // diagnostics only (tools/salu_lines.py: -gline-tables-only); the options
    // are part of the cache key, so such objects never stand in for the product's
    if (const char* e = std::getenv("PRIMEUNCORE_JIT_EXTRA"); e && *e) {
        std::string s = e;
        for (size_t i = 0; i < s.size();) {
            const size_t j = s.find(' ', i);
            const std::string w = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
            if (!w.empty()) o.push_back(w);
            if (j == std::string::npos) break;
            i = j + 1;
        }
    }
    return o;
}

int compile(const std::string& geo_src, const std::vector<std::string>& opts, std::vector<char>* code,
            std::string* log) {
    std::string main_src;
    std::vector<const char*> hnames, htexts;
    for (int i = 0; i < pu_jit_nsrc; i++) {
        const std::string n = pu_jit_src_name[i];
        if (n == "engine.hip") main_src = pu_jit_src_text[i];
        else {
            hnames.push_back(pu_jit_src_name[i]);
            htexts.push_back(pu_jit_src_text[i]);
        }
    }
    hnames.push_back("pu_jit_geo.h");
    htexts.push_back(geo_src.c_str());
    hnames.push_back("stdint.h");
    htexts.push_back(kStdint);
    hnames.push_back("stddef.h");
    htexts.push_back(kStddef);
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, main_src.c_str(), "engine.hip", (int)hnames.size(), htexts.data(),
                            hnames.data()) != HIPRTC_SUCCESS) {
        *log = "hiprtcCreateProgram failed";
        return -1;
    }
    std::vector<const char*> ov;
    for (const auto& s : opts) ov.push_back(s.c_str());
    hiprtcResult r = hiprtcCompileProgram(prog, (int)ov.size(), ov.data());
    size_t ls = 0;
    if (hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
        log->resize(ls);
        hiprtcGetProgramLog(prog, &(*log)[0]);
    }
    if (r != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return -1;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code->resize(cs);
    if (cs) hiprtcGetCode(prog, code->data());
    hiprtcDestroyProgram(&prog);
    return cs ? 0 : -1;
}

// The offline compiler (the ROCm driver, hipcc): PRIMEUNCORE_JIT_HIPCC, else
// $ROCM_PATH/bin/hipcc; "0" turns it off.  Empty when absent.
std::string offline_cc() {
    const char* e = std::getenv("PRIMEUNCORE_JIT_HIPCC");
    if (e && std::strcmp(e, "0") == 0) return "";
    std::string p;
    if (e && *e) {
        p = e;
    } else {
        const char* r = std::getenv("ROCM_PATH");
        p = std::string(r && *r ? r : "/opt/rocm") + "/bin/hipcc";
    }
    return ::access(p.c_str(), X_OK) == 0 ? p : "";
}

// Set once this library touches HIP (pu_create, the unit hooks, jit_load,
// device_arch): from then on nothing is compiled by starting another program,
// only by hipRTC in-process (a process that has initialised the GPU starts no
// compiler).  The library cannot see HIP use by others in the process (torch,
// another library), so the offline compiler is also opt-in: only a process
// that sets PRIMEUNCORE_JIT_OFFLINE=1 (tools/jit_warm.py, which never touches
// the GPU) starts it.
std::atomic<bool> g_gpu_used{false};
bool offline_allowed() {
    const char* e = std::getenv("PRIMEUNCORE_JIT_OFFLINE");
    return e && e[0] == '1' && !g_gpu_used;
}

// The offline compiler's identity for the cache key: the resolved driver and
// clang paths with their sizes, and the ROCm version file — no child process
// (jit_key also runs in processes that use the GPU).
const std::string& offline_cc_identity() {
    static const std::string id = [] {
        std::string s;
        auto add = [&](const std::string& path) {
            char rp[PATH_MAX];
            struct stat st;
            if (path.empty() || !::realpath(path.c_str(), rp) || ::stat(rp, &st) != 0) {
                s += "|-";
                return;
            }
            // (no modification time: the GPU boxes unpack the same image with their own times)
            s += std::string("|") + rp + ":" + std::to_string((long long)st.st_size);
        };
        const std::string cc = offline_cc();
        add(cc);
        const char* r = std::getenv("ROCM_PATH");
        const std::string root = r && *r ? r : "/opt/rocm";
        add(root + "/lib/llvm/bin/clang");
        std::vector<char> v;
        if (read_file(root + "/.info/version", &v)) s += "|" + std::string(v.begin(), v.end());
        return s;
    }();
    return id;
}

// Compile with the offline compiler (a child process, never from a process
// that has initialised the GPU): the embedded sources and the configuration
// are written to a scratch directory under the names the sources include.
int compile_offline(const std::string& cc, const std::string& geo_src, const std::vector<std::string>& opts,
                    std::vector<char>* code, std::string* log) {
    const char* td = std::getenv("TMPDIR");
    std::string tmpl = std::string(td && *td ? td : "/tmp") + "/pu_jit_XXXXXX";
    std::vector<char> dbuf(tmpl.begin(), tmpl.end());
    dbuf.push_back(0);
    if (!::mkdtemp(dbuf.data())) {
        *log = "mkdtemp failed";
        return -1;
    }
    const std::string d = dbuf.data();
    std::vector<std::string> files;
    auto put = [&](const std::string& name, const char* text, size_t n) {
        files.push_back(d + "/" + name);
        std::ofstream f(files.back(), std::ios::binary);
        f.write(text, (std::streamsize)n);
        return (bool)f;
    };
    bool ok = true;
    for (int i = 0; i < pu_jit_nsrc; i++)
        ok = ok && put(pu_jit_src_name[i], pu_jit_src_text[i], std::strlen(pu_jit_src_text[i]));
    ok = ok && put("pu_jit_geo.h", geo_src.data(), geo_src.size());
    const std::string out = d + "/out.hsaco", logf = d + "/cc.log", src = d + "/engine.hip";
    files.push_back(out);
    files.push_back(logf);
    int rc = -1;
    if (ok) {
        std::vector<std::string> args = {cc};
        args.insert(args.end(), opts.begin(), opts.end());
        for (const std::string& a : {std::string("-o"), out, std::string("-x"), std::string("hip"), src})
            args.push_back(a);
        std::vector<char*> argv;
        for (auto& a : args) argv.push_back(&a[0]);
        argv.push_back(nullptr);
        posix_spawn_file_actions_t fa;
        posix_spawn_file_actions_init(&fa);
        posix_spawn_file_actions_addopen(&fa, 1, logf.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        posix_spawn_file_actions_adddup2(&fa, 1, 2);
        pid_t pid = 0;
        if (posix_spawn(&pid, cc.c_str(), &fa, nullptr, argv.data(), environ) == 0) {
            int st = 0;
            while (::waitpid(pid, &st, 0) < 0 && errno == EINTR) {}
            if (WIFEXITED(st) && WEXITSTATUS(st) == 0 && read_file(out, code) && !code->empty()) rc = 0;
        } else {
            *log = "could not start " + cc;
        }
        posix_spawn_file_actions_destroy(&fa);
        if (rc != 0) {
            std::vector<char> l;
            if (read_file(logf, &l)) log->append(l.begin(), l.end());
        }
    }
    for (const auto& f : files) std::remove(f.c_str());
    ::rmdir(d.c_str());
    return rc;
}

std::mutex g_jit_mu;   // one compile at a time per process (hipRTC holds a lot of memory)
std::mutex g_mods_mu;  // the loaded modules (jit_prof_read)
std::vector<hipModule_t> g_mods;
std::vector<unsigned long long> g_prof_unloaded;   // region counters of profiling modules already unloaded
constexpr const char* kBuildArch = "gfx950";   // the library's own target (Makefile ARCH)

}  // namespace

bool jit_enabled() {
    const char* e = std::getenv("PRIMEUNCORE_JIT");
    return !(e && e[0] == '0');
}

// The engine sources this library embeds, as 8 hex digits: the prefix of
// every code object name it writes (tools/jit_warm.py keeps the code objects
// whose prefix a library in the tree carries).
std::string jit_source_tag() {
    uint64_t h = fnv1a("primeuncore-jit-src");
    for (int i = 0; i < pu_jit_nsrc; i++) {
        h = fnv1a(pu_jit_src_name[i], h);
        h = fnv1a(pu_jit_src_text[i], h);
    }
    char buf[9];
    std::snprintf(buf, sizeof buf, "%08llx", (unsigned long long)(h >> 32));
    return buf;
}

void jit_note_gpu() { g_gpu_used = true; }

std::string jit_key(const Geo& g, int waves_1level, const std::string& arch, int part, int cc) {
    uint64_t h = fnv1a("primeuncore-jit-2");
    for (int i = 0; i < pu_jit_nsrc; i++) {
        h = fnv1a(pu_jit_src_name[i], h);
        h = fnv1a(pu_jit_src_text[i], h);
    }
    h = fnv1a(geo_cxx(g), h);
    for (const auto& o : options(arch, waves_1level, part, g.num_levels == 1, cc)) h = fnv1a(o, h);
    int maj = 0, min = 0;
    hiprtcVersion(&maj, &min);
    h = fnv1a(std::to_string(maj) + "." + std::to_string(min), h);
    if (cc == kJitOffline) h = fnv1a(offline_cc_identity(), h);   // a different or upgraded hipcc/clang
    char buf[17];
    std::snprintf(buf, sizeof buf, "%016llx", (unsigned long long)h);
    return jit_source_tag() + "-" + buf;
}

namespace {
int jit_waves() {
    const char* e = std::getenv("PRIMEUNCORE_JIT_WAVES");
    return e && *e ? std::atoi(e) : 0;
}

// The current device's target ("gfx950" from "gfx950:sramecc+:xnack-").
std::string device_arch() {
    g_gpu_used = true;
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return kBuildArch;
    std::string a = p.gcnArchName;
    const size_t k = a.find(':');
    return a.empty() ? std::string(kBuildArch) : a.substr(0, k);
}

// Compile configuration g for arch into the cache; 0 or -1 (log filled).
int compile_into(const Geo& g, int waves, const std::string& arch, int part, int cc, const std::string& path,
                 std::vector<char>* code, std::string* log) {
    const std::vector<std::string> opts = options(arch, waves, part, g.num_levels == 1, cc);
    const int rc = cc == kJitOffline ? compile_offline(offline_cc(), geo_cxx(g), opts, code, log)
                                     : compile(geo_cxx(g), opts, code, log);
    if (rc != 0) return -1;
    ::mkdir(cache_dir().c_str(), 0755);
    write_file_atomic(path, *code);
    return 0;
}

// Load part `part`'s kernels (f[s][part]) from a code object; false (module
// unloaded) on failure.
bool load_module(const std::vector<char>& code, int part, JitKernels* out, std::string* why) {
    hipModule_t mod = nullptr;
    if (hipModuleLoadData(&mod, code.data()) != hipSuccess) {
        *why = "the device refused the code object";
        return false;
    }
    static const char* names[4][2] = {{"pu_jit_uncore_s0_h0", "pu_jit_uncore_s0_h1"},
                                      {"pu_jit_uncore_s1_h0", "pu_jit_uncore_s1_h1"},
                                      {"pu_jit_uncore_s2_h0", nullptr},
                                      {nullptr, "pu_jit_uncore_s3_h1"}};
    for (int s = 0; s < 4; s++)
        if (names[s][part] && hipModuleGetFunction(&out->f[s][part], mod, names[s][part]) != hipSuccess) {
            (void)hipModuleUnload(mod);
            *why = std::string("the code object lacks ") + names[s][part];
            return false;
        }
    out->mod[part] = mod;
    std::lock_guard<std::mutex> lk(g_mods_mu);
    g_mods.push_back(mod);
    return true;
}

// Part `part` of configuration g: from the cache, else compiled into it, then
// loaded; false after a message (the caller falls back to the ahead-of-time
// kernels).
bool load_part(const Geo& g, int waves, const std::string& arch, int part, JitKernels* out, bool verbose,
               std::string* key_out) {
    std::vector<char> code;
    std::string log, why;
    // the offline compiler's code object (written at build time: jit_warm), else hipRTC's
    for (int cc : {kJitOffline, kJitRtc}) {
        const std::string key = jit_key(g, waves, arch, part, cc);
        const std::string path = cache_dir() + "/" + key + ".hsaco";
        if (!read_file(path, &code)) continue;
        ::utime(path.c_str(), nullptr);          // in use: tools/jit_warm.py keeps what is used
        if (load_module(code, part, out, &why)) {
            *key_out = key;
            out->cc[part] = cc;
            return true;
        }
        // a damaged or foreign cache entry: drop it (hipRTC compiles it again below)
        std::fprintf(stderr, "[primeuncore] cached code object %s: %s; compiling it again\n", path.c_str(),
                     why.c_str());
        std::remove(path.c_str());
    }
    const std::string key = jit_key(g, waves, arch, part, kJitRtc);
    const std::string path = cache_dir() + "/" + key + ".hsaco";
    *key_out = key;
    if (verbose) std::fprintf(stderr, "[primeuncore] compiling the engine for this configuration (%s)\n", key.c_str());
    if (compile_into(g, waves, arch, part, kJitRtc, path, &code, &log) != 0) {
        std::fprintf(stderr,
                     "[primeuncore] compile-time configuration unavailable (hipRTC failed); the ahead-of-time "
                     "kernels run instead:\n%s\n",
                     log.c_str());
        return false;
    }
    if (!load_module(code, part, out, &why)) {
        std::fprintf(stderr, "[primeuncore] freshly compiled code object %s: %s; the ahead-of-time kernels run "
                             "instead\n", path.c_str(), why.c_str());
        std::remove(path.c_str());
        return false;
    }
    return true;
}
}  // namespace

int jit_load(const Geo& g, JitKernels* out, bool verbose) {
    *out = JitKernels{};
    g_gpu_used = true;
    if (!jit_enabled()) return 0;
    const int waves = jit_waves();
    const std::string arch = device_arch();
    std::lock_guard<std::mutex> lk(g_jit_mu);   // one compile at a time; another thread may have built it
    std::string key[kJitParts];
    for (int part = 0; part < kJitParts; part++)
        if (!load_part(g, waves, arch, part, out, verbose, &key[part])) {
            jit_unload(out);
            return 0;
        }
    out->ok = true;
    out->key = key[0] + "+" + key[1].substr(key[1].find('-') + 1);
    return 0;
}

// Compile (or find in the cache) without loading: needs no GPU (build-time
// warm-up), so it targets the architecture the library is built for.
int jit_warm(const Geo& g, std::string* key_out) {
    const int waves = jit_waves();
    // the offline compiler when present (and this process has put nothing on
    // the GPU), else hipRTC; a part already cached under either is kept
    const bool offline = offline_allowed() && !offline_cc().empty();
    std::lock_guard<std::mutex> lk(g_jit_mu);
    int cached = 0;
    for (int part = 0; part < kJitParts; part++) {
        const std::string ko = jit_key(g, waves, kBuildArch, part, kJitOffline);
        const std::string kr = jit_key(g, waves, kBuildArch, part, kJitRtc);
        const std::string po = cache_dir() + "/" + ko + ".hsaco", pr = cache_dir() + "/" + kr + ".hsaco";
        struct stat st;
        const bool have_o = ::stat(po.c_str(), &st) == 0 && st.st_size > 0;
        const bool have_r = !have_o && ::stat(pr.c_str(), &st) == 0 && st.st_size > 0;
        if (key_out && part == 0) *key_out = have_o || offline ? ko : kr;
        if (have_o || (have_r && !offline)) {
            ::utime((have_o ? po : pr).c_str(), nullptr);   // still in use (tools/jit_warm.py prunes what is not)
            cached++;
            continue;
        }
        std::vector<char> code;
        std::string log;
        const int cc = offline ? kJitOffline : kJitRtc;
        if (compile_into(g, waves, kBuildArch, part, cc, cc == kJitOffline ? po : pr, &code, &log) != 0)
            return set_error(PU_EIO, std::string(cc == kJitOffline ? "hipcc: " : "hipRTC: ") + log);
    }
    return cached == kJitParts ? 1 : 0;
}

void jit_unload(JitKernels* k) {
    for (hipModule_t& m : k->mod) {
        if (!m) continue;
        {
            std::lock_guard<std::mutex> lk(g_mods_mu);
            for (size_t i = 0; i < g_mods.size(); i++)
                if (g_mods[i] == m) {
                    g_mods.erase(g_mods.begin() + (long)i);
                    break;
                }
            // a profiling module's counters outlive it (a handle closed before
            // the counters are read)
            hipDeviceptr_t p = nullptr;
            size_t bytes = 0;
            if (hipModuleGetGlobal(&p, &bytes, m, "g_prof") != hipSuccess || !p) {
                (void)hipGetLastError();
            } else if (hipDeviceSynchronize() == hipSuccess) {
                std::vector<unsigned long long> buf(bytes / sizeof(unsigned long long), 0);
                if (hipMemcpyDtoH(buf.data(), p, bytes) == hipSuccess) {
                    if (g_prof_unloaded.size() < buf.size()) g_prof_unloaded.resize(buf.size(), 0);
                    for (size_t i = 0; i < buf.size(); i++) g_prof_unloaded[i] += buf[i];
                }
            }
        }
        (void)hipModuleUnload(m);
        m = nullptr;
    }
    *k = JitKernels{};
}

// Diagnostics: the region counters (g_prof) of every loaded module compiled
// with -DPU_PROF (PRIMEUNCORE_JIT_EXTRA), summed; optionally cleared with the
// per-block durations.  Returns n, or 0 when no loaded module has them.
int jit_prof_read(unsigned long long* out, int n, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    std::lock_guard<std::mutex> lk(g_mods_mu);
    std::vector<unsigned long long> buf;
    bool any = !g_prof_unloaded.empty();
    for (int i = 0; i < n; i++) out[i] = (size_t)i < g_prof_unloaded.size() ? g_prof_unloaded[i] : 0;
    if (reset) g_prof_unloaded.clear();
    for (hipModule_t m : g_mods) {
        hipDeviceptr_t p = nullptr;
        size_t bytes = 0;
        if (hipModuleGetGlobal(&p, &bytes, m, "g_prof") != hipSuccess || !p) {
            (void)hipGetLastError();   // not a profiling module: leave no error behind for the caller's runtime
            continue;
        }
        any = true;
        const size_t k = bytes / sizeof(unsigned long long);
        buf.assign(k, 0);
        if (hipMemcpyDtoH(buf.data(), p, bytes) != hipSuccess) return -1;
        for (int i = 0; i < n && (size_t)i < k; i++) out[i] += buf[i];
        if (reset) {
            if (hipMemsetD8(p, 0, bytes) != hipSuccess) return -1;
            hipDeviceptr_t q = nullptr;
            if (hipModuleGetGlobal(&q, &bytes, m, "g_blk_dur") != hipSuccess) (void)hipGetLastError();
            else if (q && hipMemsetD8(q, 0, bytes) != hipSuccess) return -1;
        }
    }
    return any ? n : 0;
}

int jit_launch(const JitKernels& k, bool sliced, bool lds_headers, int nblocks, hipStream_t stream, const Geo* d_geo,
               char* arena, int replica0, const pu_req* reqs, const uint64_t* off, int32_t* delays, uint64_t* pos,
               uint64_t budget_ticks, uint32_t flags, uint32_t* sched, int nrep) {
    void* args[] = {(void*)&d_geo, (void*)&arena, (void*)&replica0, (void*)&reqs, (void*)&off,
                    (void*)&delays, (void*)&pos, (void*)&budget_ticks, (void*)&flags, (void*)&sched, (void*)&nrep};
    // latency mode (headers in LDS): two waves, the second the M/G/1 helper (engine.hip)
    hipFunction_t f = sched ? k.f[2][0] : k.f[sliced ? 1 : 0][lds_headers ? 1 : 0];
    hipError_t e = hipModuleLaunchKernel(f, (unsigned)nblocks, 1, 1,
                                         lds_headers ? 128 : 64, 1, 1, 0, stream, args, nullptr);
    return e == hipSuccess ? 0 : PU_EIO;
}

int jit_launch_resident(const JitKernels& k, hipStream_t stream, const Geo* d_geo, char* arena, int replica,
                        pu_req* stage, void* mbox, uint64_t idle_ticks, int cap) {
    if (!k.f[3][1]) return PU_EINVAL;
    const pu_req* reqs = stage;
    const uint64_t* off = reinterpret_cast<const uint64_t*>(mbox);
    int32_t* delays = nullptr;
    uint64_t* pos = nullptr;
    uint32_t flags = 0;
    uint32_t* sched = nullptr;
    void* args[] = {(void*)&d_geo, (void*)&arena, (void*)&replica, (void*)&reqs, (void*)&off,
                    (void*)&delays, (void*)&pos, (void*)&idle_ticks, (void*)&flags, (void*)&sched, (void*)&cap};
    hipError_t e = hipModuleLaunchKernel(k.f[3][1], 1, 1, 1, 128, 1, 1, 0, stream, args, nullptr);
    return e == hipSuccess ? 0 : PU_EIO;
}

int jit_occupancy(const JitKernels& k, int mode, int* blocks_per_cu, int* lds_bytes) {
    hipFunction_t f = k.f[mode == 2 ? 2 : 1][0];
    int n = 0, lds = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 64, 0) != hipSuccess) return PU_EIO;
    if (hipFuncGetAttribute(&lds, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, f) != hipSuccess) return PU_EIO;
    *blocks_per_cu = n;
    *lds_bytes = lds;
    return 0;
}

}  // namespace pu
