// mirror_check — drives include/primeuncore.hpp (the C++ UncoreManager mirror a
// prime.cpp build would use) on the GPU the way prime.cpp does, for
// tests/test_gpu_mirror.py: config from XML, NEW_THREAD -> allocCore, each
// MEM_REQUESTS message through access_msgmem (the 24-B MsgMem records of
// reference common.h:49-59), the report at the end.
//
//   mirror_check CONFIG.xml REQS.bin THREADS.txt OUT_PREFIX
// REQS.bin: pu_req records in canonical order; THREADS.txt: "prog thread" per
// core.  Writes OUT_PREFIX.delays (one message delay per line, or "halt I D"),
// OUT_PREFIX.report.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <vector>

#include "primeuncore.hpp"

int main(int argc, char** argv) {
    if (argc != 5) {
        std::fprintf(stderr, "usage: mirror_check CONFIG.xml REQS.bin THREADS.txt OUT_PREFIX\n");
        return 2;
    }
    std::vector<pu_req> reqs;
    {
        std::ifstream f(argv[2], std::ios::binary);
        pu_req r;
        while (f.read(reinterpret_cast<char*>(&r), sizeof r)) reqs.push_back(r);
    }
    std::vector<std::pair<int, int>> threads;
    {
        std::ifstream f(argv[3]);
        int p, t;
        while (f >> p >> t) threads.push_back({p, t});
    }
    try {
        pu::UncoreManager um;
        um.init_from_xml(argv[1]);
        um.getSimStartTime();
        for (auto& pt : threads) um.allocCore(pt.first, pt.second);
        std::ofstream out(std::string(argv[4]) + ".delays");
        std::vector<unsigned char> rec;
        size_t i = 0;
        while (i < reqs.size()) {
            size_t j = i + 1;
            while (j < reqs.size() && !reqs[j].batch_start) j++;
            rec.assign((j - i) * 24, 0);                       // MsgMem: bool, int, u64 addr, i64 timer
            for (size_t k = i; k < j; k++) {
                unsigned char* p = &rec[(k - i) * 24];
                p[0] = reqs[k].mem_type ? 1 : 0;
                std::memcpy(p + 8, &reqs[k].addr, 8);
                std::memcpy(p + 16, &reqs[k].timer, 8);
            }
            try {
                out << um.access_msgmem(reqs[i].core, reqs[i].prog_id, rec.data(), j - i) << "\n";
            } catch (const pu::NegativeDelay& e) {
                out << "halt " << i + e.index << " " << e.delay << "\n";
                break;                                           // prime.cpp:133 returns
            }
            i = j;
        }
        um.getSimFinishTime();
        std::ofstream rep(std::string(argv[4]) + ".report");
        um.report(&rep);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "mirror_check: %s\n", e.what());
        return 1;
    }
    return 0;
}
