// Host check of csrc/mev_nsort.h (the device's neighbour order) and of the oracle's
// restatement (oracle/marl_oracle.c orc_std_sort_perm) against this image's
// libstdc++ std::sort, which the reference build links (cpp/IntersectionEnv.cpp:490).
// Inputs: random distances drawn from small value sets (many exact ties), continuous
// ones, sorted / reversed / constant / organ-pipe arrays, and McIlroy's adversary
// against this very std::sort, which drives it past 2*lg(n) levels into heapsort.
// Built and run by tests/test_nsort.py.  Exit status 1 on any mismatch.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <limits>
#include <random>
#include <vector>

static long g_heap = 0;
#define MEV_NS_COUNT_HEAP g_heap
#include "mev_nsort.h"

extern "C" void orc_std_sort_perm(const float* d, int n, int* perm);

struct Arr {
    std::vector<mev::NRef> v;
    mev::NRef get(int i) const { return v[i]; }
    void set(int i, mev::NRef r) { v[i] = r; }
};
struct Stk {
    std::vector<int> s;
    void push(int w) { s.push_back(w); }
    int pop() { int w = s.back(); s.pop_back(); return w; }
    int size() const { return (int)s.size(); }
};

static std::vector<int> ref_sort(const std::vector<float>& d) {
    struct NR { float dist; int id; };
    std::vector<NR> a;
    for (size_t k = 0; k < d.size(); ++k) a.push_back({d[k], (int)k});
    std::sort(a.begin(), a.end(), [](const NR& x, const NR& y) { return x.dist < y.dist; });
    std::vector<int> ids;
    for (auto& x : a) ids.push_back(x.id);
    return ids;
}

static long g_bad = 0, g_cases = 0;

static void check(const std::vector<float>& d, const char* tag) {
    const int n = (int)d.size();
    ++g_cases;
    const std::vector<int> ref = ref_sort(d);
    // the whole sort: the partitions, then a stable order of P
    Arr a;
    for (int k = 0; k < n; ++k) a.v.push_back({d[k], k});
    Stk st;
    mev::ns_introsort(a, n, std::numeric_limits<float>::infinity(), st);
    std::stable_sort(a.v.begin(), a.v.end(), [](const mev::NRef& x, const mev::NRef& y) { return x.d < y.d; });
    bool ok = true;
    for (int k = 0; k < n; ++k) ok = ok && a.v[k].id == ref[k];
    // the pruned top 5, as the device runs it
    std::vector<float> s = d;
    std::sort(s.begin(), s.end());
    const float dlim = n >= 5 ? s[4] : (n ? s[n - 1] : 0.0f);
    Arr b;
    for (int k = 0; k < n; ++k) b.v.push_back({d[k], k});
    Stk st2;
    mev::ns_introsort(b, n, dlim, st2);
    int top[5];
    const int nb = mev::ns_stable_top(b, n, 5, top);
    ok = ok && nb == std::min(n, 5);
    for (int k = 0; k < nb; ++k) ok = ok && top[k] == ref[k];
    // the oracle's restatement
    std::vector<int> perm(n > 0 ? n : 1);
    orc_std_sort_perm(d.data(), n, perm.data());
    for (int k = 0; k < n; ++k) ok = ok && perm[k] == ref[k];
    if (!ok) {
        if (g_bad < 5) printf("MISMATCH %s n=%d\n", tag, n);
        ++g_bad;
    }
}

// McIlroy, "A killer adversary for quicksort" (1999), run against this std::sort.
static std::vector<float> adversary(int n) {
    std::vector<int> val(n), idx(n);
    const int gas = n;
    int nsolid = 0, candidate = 0;
    for (int k = 0; k < n; ++k) { val[k] = gas; idx[k] = k; }
    auto cmp = [&](int x, int y) {
        if (val[x] == gas && val[y] == gas) {
            if (x == candidate) val[x] = nsolid++;
            else val[y] = nsolid++;
        }
        if (val[x] == gas) candidate = x;
        else if (val[y] == gas) candidate = y;
        return val[x] < val[y];
    };
    std::sort(idx.begin(), idx.end(), cmp);
    for (int k = 0; k < n; ++k)
        if (val[k] == gas) val[k] = nsolid++;
    std::vector<float> d(n);
    for (int k = 0; k < n; ++k) d[k] = float(val[k]);
    return d;
}

int main() {
    std::mt19937 rng(12345);
    for (int n = 0; n <= 255; ++n) {
        for (int rep = 0; rep < 60; ++rep) {
            std::vector<float> d(n);
            const int alpha = 1 + (int)(rng() % 12);  // 1..12 distinct values: ties everywhere
            for (auto& x : d) x = float(rng() % alpha) * 0.5f + 100.0f;
            check(d, "ties");
            for (auto& x : d) x = std::uniform_real_distribution<float>(0.0f, 400.0f)(rng);
            check(d, "uniform");
        }
        std::vector<float> d(n);
        for (int k = 0; k < n; ++k) d[k] = float(k);
        check(d, "sorted");
        for (int k = 0; k < n; ++k) d[k] = float(n - k);
        check(d, "reversed");
        for (int k = 0; k < n; ++k) d[k] = 7.0f;
        check(d, "constant");
        for (int k = 0; k < n; ++k) d[k] = float(std::min(k, n - 1 - k) % 9);
        check(d, "organ");
        check(adversary(n), "adversary");
    }
    printf("nsort_check: %ld cases, %ld mismatches, %ld heapsort calls\n", g_cases, g_bad, g_heap);
    if (g_bad == 0 && g_heap > 0) printf("NSORT OK\n");
    return g_bad == 0 && g_heap > 0 ? 0 : 1;
}
