// prime_server.cpp — the `prime` executable's role (reference src/prime.cpp:142-233)
// with the HIP engine as the uncore and a Unix-domain socket instead of MPI.
//
//   prime_server config.xml output [--socket PATH] [--sessions N] [--device D] [--quiet]
//
// Like prime.cpp: parse the config_prime XML (xml_parser.cpp), init the uncore,
// serve until every handler has seen PROGRAM_EXITING, then write the report to
// <output>_<session> (prime.cpp:194 writes <output>_<rank>; the reference's
// single uncore is session 0).  Sessions are independent simulations sharing
// the GPU, one engine replica (one wavefront) each.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/primeuncore.h"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s config_file output_file [--socket PATH] [--sessions N] [--device D] [--quiet]\n",
                     argv[0]);
        return 1;
    }
    std::string sock = "/tmp/prime_uncore.sock";
    int sessions = 1, device = 0, verbose = 1;
    for (int i = 3; i < argc; i++) {
        if (!std::strcmp(argv[i], "--socket") && i + 1 < argc) sock = argv[++i];
        else if (!std::strcmp(argv[i], "--sessions") && i + 1 < argc) sessions = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--quiet")) verbose = 0;
        else {
            std::fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 1;
        }
    }
    pu_sim_cfg cfg;
    if (pu_config_load_xml(argv[1], &cfg) != 0) {
        std::fprintf(stderr, "XML file parse error! (%s)\n", pu_last_error());
        return 1;
    }
    pu_handle* h = pu_create(&cfg, sessions, device);
    if (!h) {
        std::fprintf(stderr, "uncore init failed: %s\n", pu_last_error());
        return 1;
    }
    pu_server_opts o;
    std::memset(&o, 0, sizeof o);
    o.socket_path = sock.c_str();
    o.report_prefix = argv[2];
    o.num_sessions = sessions;
    o.num_recv_threads = cfg.num_recv_threads;
    o.max_msg_size = cfg.max_msg_size;
    o.verbose = verbose;
    pu_server* s = pu_server_create(h, &o);
    if (!s) {
        std::fprintf(stderr, "server: %s\n", pu_last_error());
        pu_destroy(h);
        return 1;
    }
    if (verbose) std::printf("[PriME] serving %d session(s) on %s\n", sessions, sock.c_str());
    std::fflush(stdout);
    int rc = pu_server_run(s);
    pu_server_stats st;
    pu_server_get_stats(s, &st);
    if (verbose)
        std::printf("[PriME] done: %llu messages, %llu requests in %llu launches\n", (unsigned long long)st.messages,
                    (unsigned long long)st.requests, (unsigned long long)st.launches);
    pu_server_destroy(s);
    pu_destroy(h);
    if (rc) std::fprintf(stderr, "server: %s\n", pu_last_error());
    return rc ? 1 : 0;
}
