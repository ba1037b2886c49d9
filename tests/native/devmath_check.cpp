// Host-side bit-exactness check of csrc/mev_math.h against this image's glibc libm.
// Built and run by tests/test_devmath.py (strided mode) and by hand in
// exhaustive mode:  ./devmath_check exhaustive
// Every mismatch is counted; exit status 1 if any function mismatches.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <cmath>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "mev_math.h"

static uint32_t f2u_(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f_(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static bool same(float a, float b) { return f2u_(a) == f2u_(b) || (a != a && b != b); }

template <class F>
static uint64_t parallel_range(uint32_t lo, uint32_t hi, uint32_t stride, F fn) {
    const int T = std::max(1u, std::thread::hardware_concurrency());
    std::atomic<uint64_t> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            uint64_t b = 0;
            for (uint64_t u = uint64_t(lo) + uint64_t(t) * stride; u <= hi; u += uint64_t(T) * stride) b += fn(uint32_t(u));
            bad += b;
        });
    for (auto& x : th) x.join();
    return bad.load();
}

// Evaluate over both signs of every float with |x| <= bound (bit pattern sweep).
template <class F>
static uint64_t sweep_abs(float bound, uint32_t stride, F fn) {
    const uint32_t top = f2u_(bound);
    return parallel_range(0, top, stride, [&](uint32_t u) -> uint64_t {
        return fn(u2f_(u)) + fn(u2f_(u | 0x80000000u));
    });
}

int main(int argc, char** argv) {
    const bool exhaustive = argc > 1 && std::string(argv[1]) == "exhaustive";
    const uint32_t stride = exhaustive ? 1 : 61;  // strided: ~36M args per sweep
    int rc = 0;
    auto report = [&](const char* name, uint64_t bad, uint64_t total) {
        printf("%-28s mismatches %llu / ~%llu\n", name, (unsigned long long)bad, (unsigned long long)total);
        if (bad) rc = 1;
    };

    // sincosf: |x| <= 8 covers heading (|h| <= pi) + beam offsets (|rel| <= pi).
    for (int fma_mode = 0; fma_mode < 2; ++fma_mode) {
        uint64_t bad = sweep_abs(8.0f, stride, [&](float x) -> uint64_t {
            float s, c, rs, rc2;
            if (fma_mode) mev::sincosf_impl<true>(x, &s, &c);
            else mev::sincosf_impl<false>(x, &s, &c);
            ::sincosf(x, &rs, &rc2);
            return (!same(s, rs) || !same(c, rc2)) ? 1 : 0;
        });
        report(fma_mode ? "sincosf[fma] |x|<=8" : "sincosf[nofma] |x|<=8", bad, 2ull * f2u_(8.0f) / stride);
    }
    // the single-path variant the kernels use (every |x| < 120 takes it); the
    // host glibc is the FMA build, so the generic build is compared where the two
    // builds agree (|x| <= 8)
    for (int fma_mode = 0; fma_mode < 2; ++fma_mode) {
        const float bound = fma_mode ? 120.0f : 8.0f;
        uint64_t bad = sweep_abs(bound, stride, [&](float x) -> uint64_t {
            float s, c, rs, rc2;
            if (fma_mode) mev::sincosf_reduced_impl<true>(x, &s, &c);
            else mev::sincosf_reduced_impl<false>(x, &s, &c);
            ::sincosf(x, &rs, &rc2);
            return (!same(s, rs) || !same(c, rc2)) ? 1 : 0;
        });
        report(fma_mode ? "sincosf_reduced[fma] |x|<=120" : "sincosf_reduced[nofma] |x|<=8", bad,
               2ull * f2u_(bound) / stride);
    }
    // separate sinf/cosf calls agree with sincosf (the reference calls them separately)
    report("sinf/cosf vs mev |x|<=8", sweep_abs(8.0f, stride * 7, [&](float x) -> uint64_t {
        float s, c;
        mev::sincosf(x, &s, &c);
        return (!same(s, ::sinf(x)) || !same(c, ::cosf(x))) ? 1 : 0;
    }), 2ull * f2u_(8.0f) / (stride * 7));
    // large-argument path (set_state may inject any heading)
    report("sincosf 8<|x|<=1e6", sweep_abs(1e6f, stride * 13, [&](float x) -> uint64_t {
        if (fabsf(x) <= 8.0f) return 0;
        float s, c, rs, rc2;
        mev::sincosf(x, &s, &c);
        ::sincosf(x, &rs, &rc2);
        return (!same(s, rs) || !same(c, rc2)) ? 1 : 0;
    }), 2ull * f2u_(1e6f) / (stride * 13));

    // tanf: steering angle; |x| <= 4 (beyond MAX_STEER, unclipped inputs) + large
    report("tanf |x|<=4", sweep_abs(4.0f, stride, [&](float x) -> uint64_t {
        return same(mev::tanf(x), ::tanf(x)) ? 0 : 1;
    }), 2ull * f2u_(4.0f) / stride);
    report("tanf |x|<=1e5", sweep_abs(1e5f, stride * 13, [&](float x) -> uint64_t {
        return same(mev::tanf(x), ::tanf(x)) ? 0 : 1;
    }), 2ull * f2u_(1e5f) / (stride * 13));

    // atanf over every finite float
    report("atanf all", sweep_abs(u2f_(0x7f800000u), stride, [&](float x) -> uint64_t {
        return same(mev::atanf(x), ::atanf(x)) ? 0 : 1;
    }), 2ull * 0x7f800000ull / stride);

    // the branch-free forms (wave code): atanf_bf over every float, atan2f_bf wherever
    // atan2f_special does not send the wave to atan2f
    report("atanf_bf all", sweep_abs(u2f_(0x7fffffffu), stride, [&](float x) -> uint64_t {
        return same(mev::atanf_bf(x), ::atanf(x)) ? 0 : 1;
    }), 2ull * 0x7fffffffull / stride);
    {
        const uint64_t N = exhaustive ? 2000000000ull : 40000000ull;
        const int T = std::max(1u, std::thread::hardware_concurrency());
        std::atomic<uint64_t> bad{0}, cov{0};
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(4321 + t);
                std::uniform_real_distribution<float> big(-1200.0f, 1200.0f), small(-2.0f, 2.0f);
                std::uniform_int_distribution<uint32_t> bits;
                uint64_t b = 0, c = 0;
                for (uint64_t k = t; k < N; k += T) {
                    float y, x;
                    switch (k % 5) {
                        case 0: y = big(rng); x = big(rng); break;
                        case 1: y = small(rng); x = small(rng); break;
                        case 2: y = big(rng); x = small(rng) * 1e-3f; break;
                        case 3: y = small(rng); x = (k & 8) ? 1.0f : -1.0f; break;
                        default: y = u2f_(bits(rng)); x = u2f_(bits(rng)); break;
                    }
                    if (mev::atan2f_special(y, x)) {
                        c += (x == 0.0f || y == 0.0f || std::isinf(x) || std::isinf(y) || x != x || y != y) ? 0 : 1;
                        continue;
                    }
                    if (!same(mev::atan2f_bf(y, x), ::atan2f(y, x))) {
                        if (b < 4)
                            std::printf("  atan2f_bf(%a, %a) = %a, glibc %a\n", y, x, mev::atan2f_bf(y, x),
                                        ::atan2f(y, x));
                        ++b;
                    }
                }
                bad += b;
                cov += c;
            });
        for (auto& x : th) x.join();
        report("atan2f_bf random", bad, N);
        report("atan2f_special only specials", cov, N);
    }

    // atan2f / hypotf: random pairs at simulator scales plus special values
    {
        const uint64_t N = exhaustive ? 2000000000ull : 40000000ull;
        const int T = std::max(1u, std::thread::hardware_concurrency());
        std::atomic<uint64_t> bad_a{0}, bad_h{0};
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(1234 + t);
                std::uniform_real_distribution<float> big(-1200.0f, 1200.0f), small(-2.0f, 2.0f);
                std::uniform_int_distribution<uint32_t> bits;
                uint64_t ba = 0, bh = 0;
                for (uint64_t k = t; k < N; k += T) {
                    float y, x;
                    switch (k % 4) {
                        case 0: y = big(rng); x = big(rng); break;
                        case 1: y = small(rng); x = small(rng); break;
                        case 2: y = big(rng); x = small(rng) * 1e-3f; break;
                        default: y = u2f_(bits(rng)); x = u2f_(bits(rng)); break;
                    }
                    if (!same(mev::atan2f(y, x), ::atan2f(y, x))) ++ba;
                    if ((k % 4) != 3 && !same(mev::hypotf(y, x), ::hypotf(y, x))) ++bh;
                }
                bad_a += ba;
                bad_h += bh;
            });
        for (auto& x : th) x.join();
        report("atan2f random", bad_a, N);
        report("hypotf random", bad_h, N);
        // special values
        const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-45f, -1e-45f, 3e38f, -3e38f};
        uint64_t bs = 0;
        for (float a : sp)
            for (float b : sp) bs += same(mev::atan2f(a, b), ::atan2f(a, b)) ? 0 : 1;
        report("atan2f specials", bs, 121);
    }

    // fmodf: the wrap pattern fmodf(a + PI, 2PI) for |a| <= 64, plus random pairs
    {
        const float PI_F = 3.14159265358979323846f;
        report("fmodf wrap |a|<=64", sweep_abs(64.0f, stride, [&](float a) -> uint64_t {
            return same(mev::fmodf(a + PI_F, 2.0f * PI_F), ::fmodf(a + PI_F, 2.0f * PI_F)) ? 0 : 1;
        }), 2ull * f2u_(64.0f) / stride);
        report("fmodf |x|<=1e6, y=2pi", sweep_abs(1e6f, stride * 5, [&](float a) -> uint64_t {
            return same(mev::fmodf(a, 2.0f * PI_F), ::fmodf(a, 2.0f * PI_F)) ? 0 : 1;
        }), 2ull * f2u_(1e6f) / (stride * 5));
        std::mt19937 rng(7);
        std::uniform_int_distribution<uint32_t> bits;
        std::uniform_real_distribution<float> mag(-30.0f, 30.0f);
        uint64_t badp = 0;
        const int NP = exhaustive ? 200000000 : 5000000;
        for (int k = 0; k < NP; ++k) {  // random pairs of moderate magnitude (fast path)
            float x = std::ldexp(1.0f + (bits(rng) & 0xffff) / 65536.0f, int(mag(rng))) * ((bits(rng) & 1) ? -1.f : 1.f);
            float y = std::ldexp(1.0f + (bits(rng) & 0xffff) / 65536.0f, int(mag(rng))) * ((bits(rng) & 1) ? -1.f : 1.f);
            badp += same(mev::fmodf(x, y), ::fmodf(x, y)) ? 0 : 1;
        }
        report("fmodf random moderate pairs", badp, NP);
        uint64_t bad = 0;
        const int N = exhaustive ? 200000000 : 5000000;
        for (int k = 0; k < N; ++k) {
            float x = u2f_(bits(rng)), y = u2f_(bits(rng));
            bad += same(mev::fmodf(x, y), ::fmodf(x, y)) ? 0 : 1;
        }
        report("fmodf random bits", bad, N);
    }
    printf(rc ? "DEVMATH MISMATCH\n" : "DEVMATH OK\n");
    return rc;
}
