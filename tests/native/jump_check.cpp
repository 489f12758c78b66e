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
    std::printf("%ld\n", bad);
    return 0;
}
