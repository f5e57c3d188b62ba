// placement.cpp -- see placement.h.
#include "placement.h"

#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

namespace sgpu {

namespace {

std::vector<int> parse_list(const std::string& s)
{
    std::vector<int> out;
    std::stringstream ss(s);
    std::string part;
    while (std::getline(ss, part, ',')) {
        if (part.empty() || !std::isdigit((unsigned char)part[0]))
            continue;
        const size_t dash = part.find('-');
        const int a = std::atoi(part.c_str());
        const int b = dash == std::string::npos ? a : std::atoi(part.c_str() + dash + 1);
        for (int c = a; c <= b; ++c)
            out.push_back(c);
    }
    return out;
}

std::string read_line(const std::string& path)
{
    std::ifstream f(path);
    std::string s;
    if (f)
        std::getline(f, s);
    return s;
}

// CPUs the cgroup quota pays for (cgroup v2 cpu.max "quota period"), 0 = no limit
unsigned quota_cpus()
{
    const std::string s = read_line("/sys/fs/cgroup/cpu.max");
    long q = 0, p = 0;
    if (std::sscanf(s.c_str(), "%ld %ld", &q, &p) == 2 && q > 0 && p > 0)
        return (unsigned)std::max(1L, q / p);
    return 0;
}

} // namespace

std::vector<int> place_near_device(const char* pciBusId, unsigned slice, unsigned want)
{
    std::vector<int> cpus;
    const char* env = std::getenv("SIAMESE_AMD_CPUS");
    if (env && std::strcmp(env, "none") == 0)
        return {};
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
        return {};
    if (env && *env) {
        cpus = parse_list(env);
    } else {
        std::string bus = pciBusId ? pciBusId : "";
        for (char& c : bus)
            c = (char)std::tolower((unsigned char)c);
        const std::string node = read_line("/sys/bus/pci/devices/" + bus + "/numa_node");
        const int n = node.empty() ? -1 : std::atoi(node.c_str());
        if (n < 0)
            return {};
        const std::vector<int> all =
            parse_list(read_line("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist"));
        // one logical CPU per physical core first, then their SMT siblings
        std::vector<int> primary, sibling;
        for (int c : all) {
            if (c >= CPU_SETSIZE || !CPU_ISSET(c, &allowed))
                continue;
            const std::vector<int> sib = parse_list(read_line(
                "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list"));
            (sib.empty() || sib[0] == c ? primary : sibling).push_back(c);
        }
        primary.insert(primary.end(), sibling.begin(), sibling.end());
        const unsigned q = quota_cpus();
        if (q && want > q)
            want = q;
        if (primary.empty() || want == 0)
            return {};
        const size_t total = primary.size();
        const size_t first = ((size_t)slice * want) % total;
        for (size_t k = 0; k < want && k < total; ++k)
            cpus.push_back(primary[(first + k) % total]);
        // The chosen cores' SMT siblings too (SIAMESE_AMD_SMT=0: not): more
        // logical CPUs than the quota pays for, so the library's launcher,
        // completer and assembly threads never wait for a core the stepping
        // threads hold.  Headline 4.35-4.90 vs 5.29-5.91 ms/step, 3
        // interleaved rounds on the box (profiles/r5d_smt_ab.txt).
        static const bool smt = [] {
            const char* v = std::getenv("SIAMESE_AMD_SMT");
            return !v || std::atoi(v) != 0;
        }();
        if (smt) {
            const size_t n = cpus.size();
            for (size_t k = 0; k < n; ++k) {
                const std::vector<int> sib = parse_list(read_line(
                    "/sys/devices/system/cpu/cpu" + std::to_string(cpus[k]) + "/topology/thread_siblings_list"));
                for (int c : sib)
                    if (c != cpus[k] && c < CPU_SETSIZE && CPU_ISSET(c, &allowed))
                        cpus.push_back(c);
            }
        }
    }
    cpu_set_t mask;
    CPU_ZERO(&mask);
    std::vector<int> used;
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) {
            CPU_SET(c, &mask);
            used.push_back(c);
        }
    if (used.empty() || sched_setaffinity(0, sizeof(mask), &mask) != 0)
        return {};
    return used;
}

} // namespace sgpu
