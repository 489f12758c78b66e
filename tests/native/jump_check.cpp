// Host check of the xoshiro256 jump-ahead matrices (qkd_rng.h) against stepping.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../qkd_ldpc_amd/csrc/qkd_rng.h"

int main() {
    long bad = 0;
    for (uint64_t chunk : {1ull, 64ull, 192ull, 256ull, 1000ull}) {
        std::vector<uint64_t> M(6 * 256 * 4);
        qkdr::xoshiro_jump_matrices(chunk, 6, M.data());
        for (uint64_t seed : {0ull, 1ull, 777ull, 0x1cac6d74bb9d6789ull}) {
            qkdr::Xoshiro256pp g;
            g.seed(seed);
            for (int lane = 0; lane < 64; ++lane) {
                uint64_t s[4] = {g.s0, g.s1, g.s2, g.s3};
                for (int b = 0; b < 6; ++b)
                    if ((lane >> b) & 1) qkdr::jump_apply(M.data() + (size_t)b * 1024, s);
                qkdr::Xoshiro256pp h;
                h.seed(seed);
                for (uint64_t k = 0; k < chunk * lane; ++k) h.next();
                if (s[0] != h.s0 || s[1] != h.s1 || s[2] != h.s2 || s[3] != h.s3) bad++;
            }
        }
    }
    // the polynomial form (the default of keygen_fast_kernel): lane l jumps
    // by x^(l * chunk) mod P; the same states as stepping
    for (uint64_t chunk : {1ull, 64ull, 192ull, 256ull, 1000ull}) {
        std::vector<uint64_t> polys(64 * 4);
        if (!qkdr::xoshiro_jump_polys(chunk, 64, polys.data())) bad += 1000;
        for (uint64_t seed : {0ull, 5ull, 777ull, 0x1cac6d74bb9d6789ull}) {
            qkdr::Xoshiro256pp h;
            h.seed(seed);
            for (int lane = 0; lane < 64; ++lane) {
                qkdr::Xoshiro256pp g;
                g.seed(seed);
                uint64_t s[4] = {g.s0, g.s1, g.s2, g.s3};
                qkdr::jump_poly_apply(polys.data() + (size_t)lane * 4, s);
                if (s[0] != h.s0 || s[1] != h.s1 || s[2] != h.s2 || s[3] != h.s3) bad++;
                for (uint64_t k = 0; k < chunk; ++k) h.next();
            }
        }
    }
    // x^k mod P by square and multiply (the two-wave generator's starts,
    // keygen_split_kernel): the same states as stepping k draws
    {
        uint64_t P[4];
        if (!qkdr::xoshiro_charpoly(P)) bad += 1000;
        for (uint64_t k : {0ull, 1ull, 2ull, 63ull, 160ull, 10241ull, 10240ull + 63ull * 81ull}) {
            uint64_t p[4];
            qkdr::poly_x_pow(k, P, p);
            for (uint64_t seed : {0ull, 777ull}) {
                qkdr::Xoshiro256pp g, h;
                g.seed(seed);
                h.seed(seed);
                uint64_t s[4] = {g.s0, g.s1, g.s2, g.s3};
                qkdr::jump_poly_apply(p, s);
                for (uint64_t j = 0; j < k; ++j) h.next();
                if (s[0] != h.s0 || s[1] != h.s1 || s[2] != h.s2 || s[3] != h.s3) bad++;
            }
        }
    }
    // the generator's published jump(): JUMP = x^(2^128) mod P
    {
        uint64_t P[4], r[4] = {2, 0, 0, 0};          // x
        if (!qkdr::xoshiro_charpoly(P)) bad += 1000;
        for (int k = 0; k < 128; ++k) {              // square 128 times: x^(2^128)
            uint64_t t[4];
            qkdr::poly_mulmod(r, r, P, t);
            for (int w = 0; w < 4; ++w) r[w] = t[w];
        }
        const uint64_t JUMP[4] = {0x180ec6d33cfd0abaull, 0xd5a61266f0c9392cull, 0xa9582618e03fc9aaull,
                                  0x39abdc4529b1661cull};
        for (int w = 0; w < 4; ++w)
            if (r[w] != JUMP[w]) bad += 100;
    }
    std::printf("%ld\n", bad);
    return 0;
}
