// config.cpp — config_prime XML schema loader and writer.
//
// Replaces XmlParser (reference src/xml_parser.cpp) without libxml2: a small
// element/text reader plus the reference's field semantics:
//   * //simulator, //system, //network, //directory_cache, //tlb_cache must
//     each match exactly one element (xml_parser.cpp:140, 211, 365, 447, 527);
//   * //cache must match exactly num_levels elements (xml_parser.cpp:609);
//   * required-field counts 5 / 13 / 4 / 6 / 6 / 6*num_levels
//     (xml_parser.cpp:202, 357, 437, 519, 599, 680); max_num_sharers, net_type
//     and inject_delay are optional (xml_parser.cpp:249-250, 386, 431);
//   * every field is read with `stringstream >> dec >> field`, i.e. leading
//     whitespace skipped, the longest numeric prefix converted, and the field
//     left unchanged when no number parses;
//   * defaults are the XmlParser constructor's (xml_parser.cpp:42-87).
// Missing mandatory elements make the reference dereference NULL
// (SURVEY.md §5); here they return PU_EINVAL.

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/primeuncore.h"
#include "common.h"

namespace {

struct Node {
    std::string name;
    std::string text;  // concatenated direct text children
    std::vector<int> kids;
};

struct Doc {
    std::vector<Node> nodes;
    bool ok = true;
};

// Minimal XML reader: elements, text, comments, <?...?> and <!...>
// declarations, entity &lt; &gt; &amp; &quot; &apos;.  Attributes are skipped.
class Reader {
   public:
    explicit Reader(const std::string& s) : s_(s) {}

    bool parse(Doc& d) {
        std::vector<int> stack;
        while (i_ < s_.size()) {
            if (s_[i_] == '<') {
                if (starts("<!--")) {
                    size_t e = s_.find("-->", i_ + 4);
                    if (e == std::string::npos) return false;
                    i_ = e + 3;
                } else if (starts("<?")) {
                    size_t e = s_.find("?>", i_ + 2);
                    if (e == std::string::npos) return false;
                    i_ = e + 2;
                } else if (starts("<![CDATA[")) {
                    size_t e = s_.find("]]>", i_ + 9);
                    if (e == std::string::npos) return false;
                    if (!stack.empty()) d.nodes[(size_t)stack.back()].text += s_.substr(i_ + 9, e - i_ - 9);
                    i_ = e + 3;
                } else if (starts("<!")) {
                    size_t e = s_.find('>', i_ + 2);
                    if (e == std::string::npos) return false;
                    i_ = e + 1;
                } else if (starts("</")) {
                    size_t e = s_.find('>', i_ + 2);
                    if (e == std::string::npos || stack.empty()) return false;
                    std::string nm = trim(s_.substr(i_ + 2, e - i_ - 2));
                    if (nm != d.nodes[(size_t)stack.back()].name) return false;
                    stack.pop_back();
                    i_ = e + 1;
                } else {
                    size_t e = s_.find('>', i_ + 1);
                    if (e == std::string::npos) return false;
                    std::string body = s_.substr(i_ + 1, e - i_ - 1);
                    bool self_close = !body.empty() && body.back() == '/';
                    if (self_close) body.pop_back();
                    size_t k = 0;
                    while (k < body.size() && !isspace((unsigned char)body[k])) k++;
                    Node n;
                    n.name = body.substr(0, k);
                    if (n.name.empty()) return false;
                    int id = (int)d.nodes.size();
                    d.nodes.push_back(n);
                    if (!stack.empty()) d.nodes[(size_t)stack.back()].kids.push_back(id);
                    if (!self_close) stack.push_back(id);
                    i_ = e + 1;
                }
            } else {
                size_t e = s_.find('<', i_);
                if (e == std::string::npos) e = s_.size();
                if (!stack.empty()) d.nodes[(size_t)stack.back()].text += unescape(s_.substr(i_, e - i_));
                i_ = e;
            }
        }
        return stack.empty();
    }

   private:
    bool starts(const char* p) const { return s_.compare(i_, std::strlen(p), p) == 0; }
    static std::string trim(const std::string& x) {
        size_t a = 0, b = x.size();
        while (a < b && isspace((unsigned char)x[a])) a++;
        while (b > a && isspace((unsigned char)x[b - 1])) b--;
        return x.substr(a, b - a);
    }
    static std::string unescape(const std::string& x) {
        std::string o;
        for (size_t k = 0; k < x.size(); k++) {
            if (x[k] == '&') {
                static const char* ent[5] = {"&lt;", "&gt;", "&amp;", "&quot;", "&apos;"};
                static const char rep[5] = {'<', '>', '&', '"', '\''};
                bool hit = false;
                for (int j = 0; j < 5; j++) {
                    size_t L = std::strlen(ent[j]);
                    if (x.compare(k, L, ent[j]) == 0) {
                        o += rep[j];
                        k += L - 1;
                        hit = true;
                        break;
                    }
                }
                if (!hit) o += x[k];
            } else {
                o += x[k];
            }
        }
        return o;
    }
    const std::string& s_;
    size_t i_ = 0;
};

// All elements named `name`, in document order (XPath //name).
std::vector<int> find_all(const Doc& d, const char* name) {
    std::vector<int> r;
    for (size_t i = 0; i < d.nodes.size(); i++)
        if (d.nodes[i].name == name) r.push_back((int)i);
    return r;
}

// `stringstream >> dec >> v` semantics.
template <typename T>
bool read_num(const std::string& text, T* v) {
    std::stringstream ss;
    ss << text;
    T tmp;
    ss >> std::dec >> tmp;
    if (ss.fail()) return false;
    *v = tmp;
    return true;
}

template <typename T>
void field(const Doc& d, int node, const char* name, T* dst, int* count, bool counted = true) {
    for (int k : d.nodes[(size_t)node].kids) {
        if (d.nodes[(size_t)k].name == name) {
            read_num(d.nodes[(size_t)k].text, dst);
            if (counted) (*count)++;
        }
    }
}

void cache_fields(const Doc& d, int node, pu_cache_cfg* c, int* n) {
    field(d, node, "level", &c->level, n);
    field(d, node, "share", &c->share, n);
    field(d, node, "access_time", &c->access_time, n);
    field(d, node, "size", &c->size, n);
    field(d, node, "block_size", &c->block_size, n);
    field(d, node, "num_ways", &c->num_ways, n);
}

int parse_doc(const std::string& text, pu_sim_cfg* out) {
    Doc d;
    Reader rd(text);
    if (!rd.parse(d)) return pu::set_error(PU_EINVAL, "malformed XML");
    pu_sim_cfg c;
    std::memset(&c, 0, sizeof(c));
    c.num_recv_threads = 1;  // XmlParser::XmlParser, xml_parser.cpp:45

    std::vector<int> sim = find_all(d, "simulator");
    if (sim.size() != 1) return pu::set_error(PU_EINVAL, "Error in parsing simulator structure!");
    int n = 0;
    field(d, sim[0], "max_msg_size", &c.max_msg_size, &n);
    field(d, sim[0], "num_recv_threads", &c.num_recv_threads, &n);
    field(d, sim[0], "thread_sync_interval", &c.thread_sync_interval, &n);
    field(d, sim[0], "proc_sync_interval", &c.proc_sync_interval, &n);
    field(d, sim[0], "syscall_cost", &c.syscall_cost, &n);
    if (n != 5) return pu::set_error(PU_EINVAL, "Error in parsing simulator structure!");

    std::vector<int> sys = find_all(d, "system");
    if (sys.size() != 1) return pu::set_error(PU_EINVAL, "Error in parsing system structure!");
    n = 0;
    pu_sys_cfg& y = c.sys;
    field(d, sys[0], "sys_type", &y.sys_type, &n);
    field(d, sys[0], "protocol_type", &y.protocol_type, &n);
    field(d, sys[0], "max_num_sharers", &y.max_num_sharers, &n, false);
    field(d, sys[0], "page_size", &y.page_size, &n);
    field(d, sys[0], "tlb_enable", &y.tlb_enable, &n);
    field(d, sys[0], "shared_llc", &y.shared_llc, &n);
    field(d, sys[0], "verbose_report", &y.verbose_report, &n);
    field(d, sys[0], "cpi_nonmem", &y.cpi_nonmem, &n);
    field(d, sys[0], "dram_access_time", &y.dram_access_time, &n);
    field(d, sys[0], "num_levels", &y.num_levels, &n);
    field(d, sys[0], "num_cores", &y.num_cores, &n);
    field(d, sys[0], "bus_latency", &y.bus_latency, &n);
    field(d, sys[0], "page_miss_delay", &y.page_miss_delay, &n);
    field(d, sys[0], "freq", &y.freq, &n);
    if (n != 13) return pu::set_error(PU_EINVAL, "Error in parsing system structure!");
    if (y.num_levels < 1 || y.num_levels > PU_MAX_LEVELS)
        return pu::set_error(PU_ENOTSUP, "num_levels must be 1..4");

    std::vector<int> net = find_all(d, "network");
    if (net.size() != 1) return pu::set_error(PU_EINVAL, "Error in parsing network structure!");
    n = 0;
    field(d, net[0], "net_type", &y.network.net_type, &n, false);
    field(d, net[0], "data_width", &y.network.data_width, &n);
    field(d, net[0], "header_flits", &y.network.header_flits, &n);
    field(d, net[0], "router_delay", &y.network.router_delay, &n);
    field(d, net[0], "link_delay", &y.network.link_delay, &n);
    field(d, net[0], "inject_delay", &y.network.inject_delay, &n, false);
    if (n != 4) return pu::set_error(PU_EINVAL, "Error in parsing network structure!");

    std::vector<int> dir = find_all(d, "directory_cache");
    if (dir.size() != 1) return pu::set_error(PU_EINVAL, "Error in parsing directory cache structure!");
    n = 0;
    cache_fields(d, dir[0], &y.directory_cache, &n);
    if (n != 6) return pu::set_error(PU_EINVAL, "Error in parsing directory cache structure!");

    std::vector<int> tlb = find_all(d, "tlb_cache");
    if (tlb.size() != 1) return pu::set_error(PU_EINVAL, "Error in parsing TLB cache structure!");
    n = 0;
    cache_fields(d, tlb[0], &y.tlb_cache, &n);
    if (n != 6) return pu::set_error(PU_EINVAL, "Error in parsing TLB cache structure!");

    // optional <dram> element (pu_dram_cfg: the opt-in bank model); the
    // reference's XPath parser never looks at it
    std::vector<int> dram = find_all(d, "dram");
    if (dram.size() > 1) return pu::set_error(PU_EINVAL, "Error in parsing dram structure!");
    if (dram.size() == 1) {
        int m = 0;
        field(d, dram[0], "banks", &y.dram.banks, &m);
        field(d, dram[0], "row_bytes", &y.dram.row_bytes, &m);
        field(d, dram[0], "t_rcd", &y.dram.t_rcd, &m);
        field(d, dram[0], "t_rp", &y.dram.t_rp, &m);
        field(d, dram[0], "t_burst", &y.dram.t_burst, &m);
        if (m != 5) return pu::set_error(PU_EINVAL, "Error in parsing dram structure!");
    }

    std::vector<int> caches = find_all(d, "cache");
    if ((int)caches.size() != y.num_levels) return pu::set_error(PU_EINVAL, "Error in parsing cache structure!");
    n = 0;
    for (int i = 0; i < y.num_levels; i++) cache_fields(d, caches[(size_t)i], &y.cache[i], &n);
    if (n != 6 * y.num_levels) return pu::set_error(PU_EINVAL, "Error in parsing cache structure!");

    *out = c;
    return 0;
}

void put(std::ostringstream& o, const char* ind, const char* k, long long v) {
    o << ind << '<' << k << '>' << v << "</" << k << ">\n";
}
void putd(std::ostringstream& o, const char* ind, const char* k, double v) {
    o << ind << '<' << k << '>' << v << "</" << k << ">\n";
}
void put_cache(std::ostringstream& o, const char* ind, const char* tag, const pu_cache_cfg& c) {
    std::string in2 = std::string(ind) + "   ";
    o << ind << '<' << tag << ">\n";
    put(o, in2.c_str(), "level", c.level);
    put(o, in2.c_str(), "share", c.share);
    put(o, in2.c_str(), "access_time", c.access_time);
    put(o, in2.c_str(), "size", (long long)c.size);
    put(o, in2.c_str(), "block_size", (long long)c.block_size);
    put(o, in2.c_str(), "num_ways", (long long)c.num_ways);
    o << ind << "</" << tag << ">\n";
}

}  // namespace

extern "C" {

int pu_config_parse_xml(const char* text, size_t len, pu_sim_cfg* out) {
    if (!text || !out) return pu::set_error(PU_EINVAL, "null argument");
    return parse_doc(std::string(text, len), out);
}

int pu_config_load_xml(const char* path, pu_sim_cfg* out) {
    if (!path || !out) return pu::set_error(PU_EINVAL, "null argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return pu::set_error(PU_EINVAL, std::string("cannot open ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse_doc(ss.str(), out);
}

// Layout of tools/config_prime's writer (config_prime:39-54, 202-216).
int pu_config_write_xml(const pu_sim_cfg* c, char* buf, size_t cap, size_t* written) {
    if (!c) return pu::set_error(PU_EINVAL, "null config");
    std::ostringstream o;
    const pu_sys_cfg& y = c->sys;
    o << "<?xml version = \"1.0\" encoding = \"utf-8\" standalone = \"yes\"?>\n\n";
    o << "<simulator>\n";
    const char* i1 = "    ";
    const char* i2 = "       ";
    const char* i3 = "          ";
    put(o, i1, "max_msg_size", c->max_msg_size);
    put(o, i1, "thread_sync_interval", c->thread_sync_interval);
    put(o, i1, "proc_sync_interval", c->proc_sync_interval);
    put(o, i1, "syscall_cost", c->syscall_cost);
    put(o, i1, "num_recv_threads", c->num_recv_threads);
    o << i1 << "<system>\n";
    put(o, i2, "dram_access_time", y.dram_access_time);
    put(o, i2, "num_levels", y.num_levels);
    putd(o, i2, "cpi_nonmem", y.cpi_nonmem);
    put(o, i2, "num_cores", y.num_cores);
    put(o, i2, "sys_type", y.sys_type);
    put(o, i2, "protocol_type", y.protocol_type);
    put(o, i2, "max_num_sharers", y.max_num_sharers);
    put(o, i2, "page_size", y.page_size);
    put(o, i2, "tlb_enable", y.tlb_enable);
    put(o, i2, "shared_llc", y.shared_llc);
    put(o, i2, "verbose_report", y.verbose_report);
    putd(o, i2, "freq", y.freq);
    put(o, i2, "bus_latency", y.bus_latency);
    put(o, i2, "page_miss_delay", y.page_miss_delay);
    o << i2 << "<network>\n";
    put(o, i3, "net_type", y.network.net_type);
    put(o, i3, "data_width", y.network.data_width);
    put(o, i3, "header_flits", y.network.header_flits);
    put(o, i3, "router_delay", (long long)y.network.router_delay);
    put(o, i3, "link_delay", (long long)y.network.link_delay);
    put(o, i3, "inject_delay", (long long)y.network.inject_delay);
    o << i2 << "</network>\n";
    for (int i = 0; i < y.num_levels && i < PU_MAX_LEVELS; i++) put_cache(o, i2, "cache", y.cache[i]);
    put_cache(o, i2, "directory_cache", y.directory_cache);
    put_cache(o, i2, "tlb_cache", y.tlb_cache);
    if (y.dram.banks > 0) {   // the opt-in bank model only; reference configs stay config_prime's layout
        o << i2 << "<dram>\n";
        put(o, i3, "banks", y.dram.banks);
        put(o, i3, "row_bytes", (long long)y.dram.row_bytes);
        put(o, i3, "t_rcd", y.dram.t_rcd);
        put(o, i3, "t_rp", y.dram.t_rp);
        put(o, i3, "t_burst", y.dram.t_burst);
        o << i2 << "</dram>\n";
    }
    o << i1 << "</system>\n";
    o << "</simulator>\n";
    std::string s = o.str();
    if (written) *written = s.size();
    if (buf && cap) {
        size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
        if (s.size() >= cap) return PU_ERANGE;
    }
    return 0;
}

}  // extern "C"
