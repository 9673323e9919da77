// Host build of csrc/exact_math.hpp for tests/test_exact_math.py: reads
// n (y, x) f64 pairs from argv[1], writes n (atan2_cr, glibc atan2) pairs to
// argv[2].  Compiled with g++ -ffp-contract=off -DACM_HD= (no HIP).
#include <cmath>
#include <cstdio>
#include <vector>

#include "exact_math.hpp"

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    std::vector<double> in;
    double buf[2];
    while (std::fread(buf, sizeof(double), 2, f) == 2) {
        in.push_back(buf[0]);
        in.push_back(buf[1]);
    }
    std::fclose(f);
    std::vector<double> out(in.size());
    for (size_t i = 0; i < in.size(); i += 2) {
        out[i] = acm::xm::atan2_cr(in[i], in[i + 1]);
        out[i + 1] = std::atan2(in[i], in[i + 1]);
    }
    FILE* g = std::fopen(argv[2], "wb");
    if (!g) return 4;
    std::fwrite(out.data(), sizeof(double), out.size(), g);
    std::fclose(g);
    return 0;
}
