// qkd_rng.h — key-pair generation for one QKD trial, host and device.
//
// Reproduces the reference's per-trial key pair bit for bit:
//   run_trial (reference src/simulation.cpp:161-168):
//     Xoshiro256PlusPlus prng(seed);                         (XoshiroCpp 1.1)
//     generate_random_bit_array(prng, N, alice);             (array_and_matrix_operations.cpp:424-431)
//     q = introduce_errors(prng, alice, N, q_nom, bob);      (array_and_matrix_operations.cpp:434-460)
//
// Third-party algorithms restated (published, absent from the reference tree):
//   * SplitMix64 seeding + xoshiro256++ (XoshiroCpp 1.1).
//   * libstdc++ 11 uniform_int_distribution for a 64-bit engine: Lemire's
//     multiply-shift with rejection (_S_nd, 128-bit product). For {0,1} it is
//     exactly `draw >> 63` (threshold 0, never rejects).
//   * libstdc++ 11 std::shuffle: for an even length, one lone swap of
//     position 1 with {0,1}; then pairs (i, i+1) from one draw x in
//     [0, (i+1)(i+2)): swap(i, x / (i+2)), swap(i+1, x % (i+2)).
//
// The reference materialises and shuffles a size_t[N] position array and then
// flips bob[pos[p]] for p < ne = floor(N*q). Only pos[0..ne) matters, and this
// forward shuffle never moves an element INTO a low position except as
// "pos[x] = i" (the step index i). So the whole shuffle reduces to:
//   steps i < ne:  low[i] = low[x]; low[x] = i      (exact simulation, ne slots)
//   steps i >= ne: if (x < ne) low[x] = i            (last writer wins)
// which needs ne words of scratch instead of N, with identical results.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define QKD_RHD __host__ __device__ __forceinline__
#else
#define QKD_RHD inline
#endif

namespace qkdr {

struct Xoshiro256pp {
    uint64_t s0, s1, s2, s3;

    QKD_RHD static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

    QKD_RHD void seed(uint64_t seed) {
        uint64_t z = seed;
        uint64_t w[4];
        for (int i = 0; i < 4; ++i) {
            z += 0x9e3779b97f4a7c15ull;
            uint64_t v = z;
            v = (v ^ (v >> 30)) * 0xbf58476d1ce4e5b9ull;
            v = (v ^ (v >> 27)) * 0x94d049bb133111ebull;
            w[i] = v ^ (v >> 31);
        }
        s0 = w[0]; s1 = w[1]; s2 = w[2]; s3 = w[3];
    }

    QKD_RHD uint64_t next() {
        const uint64_t r = rotl(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        s2 ^= s0;
        s3 ^= s1;
        s1 ^= s2;
        s0 ^= s3;
        s2 ^= t;
        s3 = rotl(s3, 45);
        return r;
    }

#if defined(__HIP_DEVICE_COMPILE__)
    // next() for gfx950's 32-bit lanes: each 64-bit rotate as two
    // v_alignbit_b32 (funnel shifts) and each pair of chained XORs as one
    // v_bitop3_b32 per half (s1 ^ s2 ^ s0, s0 ^ s3 ^ s1, s2 ^ s0 ^ t: the same
    // values next() leaves), 18 operations a draw instead of ~24.
    static __device__ __forceinline__ uint64_t rotl_d(uint64_t x, int k) {   // 0 < k < 64, k != 32
        const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        const uint32_t j = k < 32 ? 32u - (uint32_t)k : 64u - (uint32_t)k;
        const uint32_t a = __builtin_amdgcn_alignbit(hi, lo, j), b = __builtin_amdgcn_alignbit(lo, hi, j);
        return k < 32 ? ((uint64_t)a << 32) | b : ((uint64_t)b << 32) | a;
    }
    static __device__ __forceinline__ uint64_t xor3_d(uint64_t a, uint64_t b, uint64_t c) {
        const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, (unsigned char)0x96);
        const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32),
                                                        (unsigned char)0x96);
        return ((uint64_t)hi << 32) | lo;
    }
    __device__ __forceinline__ uint64_t next_fast() {
        const uint64_t r = rotl_d(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        const uint64_t n1 = xor3_d(s1, s2, s0);
        const uint64_t n0 = xor3_d(s0, s3, s1);
        const uint64_t n2 = xor3_d(s2, s0, t);
        s3 = rotl_d(s3 ^ s1, 45);
        s0 = n0;
        s1 = n1;
        s2 = n2;
        return r;
    }
#else
    uint64_t next_fast() { return next(); }
#endif
};

QKD_RHD uint64_t mul_hi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// uniform_int_distribution<size_t>{0, range-1}(g) with a full-range 64-bit g.
QKD_RHD uint64_t lemire(Xoshiro256pp& g, uint64_t range) {
    uint64_t d = g.next();
    uint64_t low = d * range;
    if (low < range) {
        const uint64_t thr = (0 - range) % range;
        while (low < thr) {
            d = g.next();
            low = d * range;
        }
    }
    return mul_hi64(d, range);
}

// floor(N * q) as the reference computes it: static_cast<size_t>(N * q).
QKD_RHD uint64_t num_errors(uint32_t n, double q) {
    const double v = (double)n * q;
    return v <= 0.0 ? 0 : (uint64_t)v;
}

// Shuffle-and-track: fills low[0..ne) with the positions that the reference's
// shuffled array holds at indices [0, ne). `low` is caller scratch of ne words.
// Consumes draws from g exactly as std::shuffle does.
template <typename LowT>
QKD_RHD void shuffle_low_positions(Xoshiro256pp& g, uint32_t n, uint32_t ne, LowT* low) {
    for (uint32_t p = 0; p < ne; ++p) low[p] = p;
    if (n <= 1) return;
    uint32_t i = 1;
    auto step = [&](uint32_t step_i, uint32_t x) {
        if (step_i < ne) {
            LowT v = low[x];          // x <= step_i < ne
            low[x] = step_i;
            low[step_i] = v;
        } else if (x < ne) {
            low[x] = step_i;
        }
    };
    if ((n & 1u) == 0) {                              // even length: lone first swap
        const uint32_t x = (uint32_t)(g.next() >> 63);  // uniform {0,1}
        step(1, x);
        i = 2;
    }
    while (i < n) {
        const uint64_t b1 = (uint64_t)i + 2;
        const uint64_t x = lemire(g, ((uint64_t)i + 1) * b1);
        // x < (i+1)(i+2) < 2^64; both quotient and remainder fit 32 bits for n < 2^31.
        const uint32_t a = (uint32_t)(x / b1);
        const uint32_t b = (uint32_t)(x - (uint64_t)a * b1);
        step(i, a);
        step(i + 1, b);
        i += 2;
    }
}

// ---------------------------------------------------------------------------
// Jump-ahead for the parallel key generator (decode.hip: keygen_fast_kernel).
//
// xoshiro256's state transition (next() without its output scrambler) is
// linear over GF(2)^256, so "advance by j draws" is a 256x256 bit matrix T^j.
// A matrix is stored as 256 columns of 4 words: column k is the image of the
// unit state with bit k set (bits 0..63 = s0, ..., 192..255 = s3).
// ---------------------------------------------------------------------------

QKD_RHD void xoshiro_step_state(uint64_t s[4]) {
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = (s[3] << 45) | (s[3] >> 19);
}

// s <- M s
QKD_RHD void jump_apply(const uint64_t* cols, uint64_t s[4]) {
    uint64_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
    for (int w = 0; w < 4; ++w) {
        const uint64_t sw = s[w];
        const uint64_t* c = cols + (size_t)w * 64 * 4;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 8
#endif
        for (int j = 0; j < 64; ++j) {
            const uint64_t m = (uint64_t)0 - ((sw >> j) & 1u);
            o0 ^= c[j * 4 + 0] & m;
            o1 ^= c[j * 4 + 1] & m;
            o2 ^= c[j * 4 + 2] & m;
            o3 ^= c[j * 4 + 3] & m;
        }
    }
    s[0] = o0;
    s[1] = o1;
    s[2] = o2;
    s[3] = o3;
}

// Host: out[b] = T^(chunk * 2^b), b = 0..levels-1 (levels * 256 * 4 words).
inline void xoshiro_jump_matrices(uint64_t chunk, int levels, uint64_t* out) {
    const size_t MW = 256 * 4;
    uint64_t* T = new uint64_t[MW];
    uint64_t* R = new uint64_t[MW];
    uint64_t* tmp = new uint64_t[MW];
    for (int k = 0; k < 256; ++k) {
        uint64_t v[4] = {0, 0, 0, 0};
        v[k >> 6] = 1ull << (k & 63);
        xoshiro_step_state(v);
        for (int w = 0; w < 4; ++w) T[k * 4 + w] = v[w];
    }
    // mul(A, B) = A * B, column by column: (A B) e_k = A (B e_k)
    auto mul = [&](const uint64_t* A, const uint64_t* B, uint64_t* C) {
        for (int k = 0; k < 256; ++k) {
            uint64_t v[4] = {B[k * 4], B[k * 4 + 1], B[k * 4 + 2], B[k * 4 + 3]};
            jump_apply(A, v);
            for (int w = 0; w < 4; ++w) C[k * 4 + w] = v[w];
        }
    };
    // R = T^chunk (square and multiply)
    for (int k = 0; k < 256; ++k) {
        for (int w = 0; w < 4; ++w) R[k * 4 + w] = 0;
        R[k * 4 + (k >> 6)] = 1ull << (k & 63);
    }
    uint64_t e = chunk;
    while (e) {
        if (e & 1) {
            mul(T, R, tmp);
            for (size_t i = 0; i < MW; ++i) R[i] = tmp[i];
        }
        mul(T, T, tmp);
        for (size_t i = 0; i < MW; ++i) T[i] = tmp[i];
        e >>= 1;
    }
    for (int b = 0; b < levels; ++b) {
        for (size_t i = 0; i < MW; ++i) out[b * MW + i] = R[i];
        mul(R, R, tmp);
        for (size_t i = 0; i < MW; ++i) R[i] = tmp[i];
    }
    delete[] T;
    delete[] R;
    delete[] tmp;
}

// ---------------------------------------------------------------------------
// Jump-ahead by polynomial (the default of keygen_fast_kernel).
//
// T satisfies its characteristic polynomial P (degree 256; xoshiro256's is
// primitive), so T^k = (x^k mod P)(T): with p = x^k mod P = sum_i p_i x^i,
//   T^k s = sum_{i < 256} p_i T^i s,
// i.e. 256 state steps from s, XOR-accumulating the states whose coefficient
// is set: about 256 x (one state step + a masked 256-bit XOR) operations per
// lane, no matrix reads (the matrix form above costs 256 masked column XORs
// per jump level, with the columns streamed from memory). This is the
// construction of the generator's own published jump() (its JUMP constant is
// x^(2^128) mod P; tests/native/jump_check.cpp checks that too).
// A polynomial of degree < 256 is 4 words, bit i = coefficient of x^i; P
// itself needs bit 256 (implicit: P = x^256 + the 4 words).
// ---------------------------------------------------------------------------

// P by Berlekamp-Massey over GF(2) on 512 output bits of a linear functional
// of the state (bit 0 of s0 after each step, from a nonzero state): the
// sequence's connection polynomial C(x) = 1 + c_1 x + ... + c_L x^L has
// L = 256 for a primitive T, and P(x) = x^L C(1/x). Returns false if L != 256.
inline bool xoshiro_charpoly(uint64_t P[4]) {
    const int n = 512;
    uint8_t seq[512];
    uint64_t s[4] = {0x9e3779b97f4a7c15ull, 0x0123456789abcdefull, 0xfedcba9876543210ull, 1ull};
    for (int i = 0; i < n; ++i) {
        seq[i] = (uint8_t)(s[0] & 1u);
        xoshiro_step_state(s);
    }
    uint8_t C[513] = {0}, B[513] = {0}, Tm[513];
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int i = 0; i < n; ++i) {
        uint8_t d = seq[i];
        for (int j = 1; j <= L; ++j) d ^= (uint8_t)(C[j] & seq[i - j]);
        if (!d) {
            ++m;
            continue;
        }
        for (int j = 0; j <= n; ++j) Tm[j] = C[j];
        for (int j = 0; j + m <= n; ++j) C[j + m] ^= B[j];
        if (2 * L <= i) {
            L = i + 1 - L;
            for (int j = 0; j <= n; ++j) B[j] = Tm[j];
            m = 1;
        } else {
            ++m;
        }
    }
    if (L != 256) return false;
    P[0] = P[1] = P[2] = P[3] = 0;
    for (int i = 0; i < 256; ++i)              // coefficient of x^i in P is c_{256 - i}
        if (C[256 - i]) P[i >> 6] |= 1ull << (i & 63);
    return true;
}

// r <- r * x mod P
inline void poly_mulx_mod(uint64_t r[4], const uint64_t P[4]) {
    const uint64_t top = r[3] >> 63;
    r[3] = (r[3] << 1) | (r[2] >> 63);
    r[2] = (r[2] << 1) | (r[1] >> 63);
    r[1] = (r[1] << 1) | (r[0] >> 63);
    r[0] <<= 1;
    if (top) {
        r[0] ^= P[0];
        r[1] ^= P[1];
        r[2] ^= P[2];
        r[3] ^= P[3];
    }
}

// r <- a * b mod P (carry-less, shift-and-add over b's bits)
inline void poly_mulmod(const uint64_t a[4], const uint64_t b[4], const uint64_t P[4], uint64_t r[4]) {
    uint64_t acc[4] = {0, 0, 0, 0}, t[4] = {a[0], a[1], a[2], a[3]};
    for (int i = 0; i < 256; ++i) {
        if ((b[i >> 6] >> (i & 63)) & 1u)
            for (int w = 0; w < 4; ++w) acc[w] ^= t[w];
        poly_mulx_mod(t, P);
    }
    for (int w = 0; w < 4; ++w) r[w] = acc[w];
}

// r = x^k mod P (square and multiply).
inline void poly_x_pow(uint64_t k, const uint64_t P[4], uint64_t r[4]) {
    uint64_t acc[4] = {1, 0, 0, 0}, base[4] = {2, 0, 0, 0}, t[4];
    for (; k; k >>= 1) {
        if (k & 1u) {
            poly_mulmod(acc, base, P, t);
            for (int w = 0; w < 4; ++w) acc[w] = t[w];
        }
        poly_mulmod(base, base, P, t);
        for (int w = 0; w < 4; ++w) base[w] = t[w];
    }
    for (int w = 0; w < 4; ++w) r[w] = acc[w];
}

// out[l] = x^(l * chunk) mod P for lanes l = 0 .. lanes-1 (4 words each).
inline bool xoshiro_jump_polys(uint64_t chunk, int lanes, uint64_t* out) {
    uint64_t P[4];
    if (!xoshiro_charpoly(P)) return false;
    uint64_t step[4] = {1, 0, 0, 0};                 // x^chunk mod P
    for (uint64_t k = 0; k < chunk; ++k) poly_mulx_mod(step, P);
    uint64_t r[4] = {1, 0, 0, 0};
    for (int l = 0; l < lanes; ++l) {
        for (int w = 0; w < 4; ++w) out[(size_t)l * 4 + w] = r[w];
        uint64_t nr[4];
        poly_mulmod(r, step, P, nr);
        for (int w = 0; w < 4; ++w) r[w] = nr[w];
    }
    return true;
}

// s <- p(T) s for a jump polynomial p (4 words): 256 state steps, the states
// of the set coefficients XOR-accumulated (masks, no branches).
QKD_RHD void jump_poly_apply(const uint64_t p[4], uint64_t s[4]) {
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint64_t t[4] = {s[0], s[1], s[2], s[3]};
#if defined(__HIP_DEVICE_COMPILE__)
#if !defined(__gfx950__)
#error "qkd_rng.h: the device jump uses gfx950's v_bitop3_b32; build with --offload-arch=gfx950"
#endif
    // gfx950: a coefficient's mask is one sign-extended bit field extract
    // (v_bfe_i32), and each 32-bit half of a ^= t & m one v_bitop3_b32 (truth
    // table f(a, t, m) = a ^ (t & m) = 0xF0 ^ (0xCC & 0xAA) = 0x78)
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < 8; ++w) {
        const int pw = (int)(uint32_t)(p[w >> 1] >> (32 * (w & 1)));
#pragma unroll 8
        for (int j = 0; j < 32; ++j) {
            const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe(pw, j, 1);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                h[2 * k] = __builtin_amdgcn_bitop3_b32(h[2 * k], (uint32_t)t[k], m, (unsigned char)0x78);
                h[2 * k + 1] = __builtin_amdgcn_bitop3_b32(h[2 * k + 1], (uint32_t)(t[k] >> 32), m, (unsigned char)0x78);
            }
            xoshiro_step_state(t);
        }
    }
    a0 = ((uint64_t)h[1] << 32) | h[0];
    a1 = ((uint64_t)h[3] << 32) | h[2];
    a2 = ((uint64_t)h[5] << 32) | h[4];
    a3 = ((uint64_t)h[7] << 32) | h[6];
#else
    // over 32-bit halves of p (the device form's order)
    for (int w = 0; w < 8; ++w) {
        const uint32_t pw = (uint32_t)(p[w >> 1] >> (32 * (w & 1)));
        for (int j = 0; j < 32; ++j) {
            const uint32_t m32 = 0u - ((pw >> j) & 1u);
            const uint64_t m = ((uint64_t)m32 << 32) | m32;
            a0 ^= t[0] & m;
            a1 ^= t[1] & m;
            a2 ^= t[2] & m;
            a3 ^= t[3] & m;
            xoshiro_step_state(t);
        }
    }
#endif
    s[0] = a0;
    s[1] = a1;
    s[2] = a2;
    s[3] = a3;
}

// Draw count of one trial: N alice bits, the lone swap draw (even N), one
// Lemire draw per shuffle pair (std::shuffle, see shuffle_low_positions),
// without rejections.
QKD_RHD uint64_t trial_draws(uint32_t n) {
    return (n & 1u) == 0 ? (uint64_t)n + 1 + (n >= 2 ? (n - 2) / 2 : 0) : (uint64_t)n + (n - 1) / 2;
}

}  // namespace qkdr
