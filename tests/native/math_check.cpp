// Host build of the device math (qkd_math.h) checked against glibc, bit for bit.
// Usage: math_check <samples> <seed>; prints "<mismatches> <first-mismatch-info>".
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../qkd_ldpc_amd/csrc/qkd_math.h"

static uint64_t bits(double x) { uint64_t u; std::memcpy(&u, &x, 8); return u; }

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 g(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long bad = 0, total = 0;
    auto chk = [&](int which, double x) {
        double r, m;
        switch (which) {
            case 0: r = std::tanh(x); m = qkdm::tanh_ref(x); break;
            case 1: r = std::atanh(x); m = qkdm::atanh_ref(x); break;
            case 2: r = std::expm1(x); m = qkdm::expm1_ref(x); break;
            case 3: r = std::log1p(x); m = qkdm::log1p_ref(x); break;
            case 4: r = std::tanh(x); m = qkdm::tanh_flat(x); break;
            default: r = std::atanh(x); m = qkdm::atanh_flat(x); break;
        }
        total++;
        if (bits(r) != bits(m) && !(std::isnan(r) && std::isnan(m))) {
            if (bad == 0) printf("# f%d x=%a libm=%a mine=%a\n", which, x, r, m);
            bad++;
        }
    };
    for (long i = 0; i < n; ++i) {
        const double u = U(g);
        for (int w = 0; w < 2; ++w) {                      // path-by-path (w=0) and flat (w=1) forms
            chk(4 * w + 0, u * 60.0);                      // message range /2, beyond 22
            chk(4 * w + 0, std::ldexp(u, (int)(g() % 72) - 66));   // tiny .. 64
            chk(4 * w + 0, std::ldexp(std::round(u * 64.0), -5));  // k-boundary neighbourhoods
            chk(5 * w + 1, u);
            chk(5 * w + 1, std::ldexp(u, -(int)(g() % 60)));
            chk(5 * w + 1, std::copysign(1.0 - std::ldexp(std::fabs(u), -(int)(g() % 54)), u));
            chk(5 * w + 1, std::nextafter(std::copysign(1.0, u), 0.0));
        }
        chk(2, u * 750.0);
        chk(2, std::ldexp(u, (int)(g() % 72) - 64));
        chk(3, std::fabs(u) * 1e6);
        chk(3, std::ldexp(std::fabs(u), (int)(g() % 130) - 66));
        chk(3, u * 0.9999);
        uint64_t rb = g();
        double x;
        std::memcpy(&x, &rb, 8);
        chk(0, x); chk(1, x); chk(2, x); chk(3, x); chk(4, x); chk(5, x);
    }
    const double sp[] = {0.0, -0.0, 1.0, -1.0, 22.0, -22.0, 0.5, -0.5, INFINITY, -INFINITY, NAN,
                         0x1p-28, 0x1p-55, 0x1p-54, 709.78, 0x1.62e42fefa39efp+9, -38.0, 0.41422};
    for (double x : sp) for (int w = 0; w < 6; ++w) chk(w, x);
    // exhaustive-ish sweeps over the exponent range of both flat forms
    for (int ex = -1075; ex <= 1024; ++ex)
        for (int j = 0; j < 64; ++j) {
            const double x = std::ldexp(1.0 + j / 64.0, ex);
            for (double y : {x, -x, std::nextafter(x, 0.0), -std::nextafter(x, INFINITY)}) { chk(4, y); chk(5, y); }
        }
    printf("%ld %ld\n", bad, total);
    return 0;
}
