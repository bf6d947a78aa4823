// Host check of the data-parallel restatement of libstdc++'s introselect (the plan of the
// GPU kernel rez_ties_kernel) against std::nth_element itself, on tie-heavy keys.
//   g++ -O2 -std=c++17 tools/nth_emul.cpp -o /tmp/nth_emul && /tmp/nth_emul
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef uint64_t P;   // key << 32 | index
static inline uint32_t K(P p) { return (uint32_t)(p >> 32); }
static bool comp(const P& a, const P& b) { return K(a) > K(b); }

static void adjust_heap(P* A, int64_t f, int64_t hole, int64_t len, P value) {
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (K(A[f + second]) > K(A[f + second - 1])) second--;
        A[f + hole] = A[f + second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        A[f + hole] = A[f + second - 1];
        hole = second - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && K(A[f + parent]) > K(value)) {
        A[f + hole] = A[f + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A[f + hole] = value;
}
static void heap_select(P* A, int64_t f, int64_t m, int64_t l) {
    const int64_t len = m - f;
    if (len >= 2)
        for (int64_t parent = (len - 2) / 2;; --parent) {
            adjust_heap(A, f, parent, len, A[f + parent]);
            if (parent == 0) break;
        }
    for (int64_t i = m; i < l; ++i)
        if (K(A[i]) > K(A[f])) {
            P v = A[i];
            A[i] = A[f];
            adjust_heap(A, f, 0, len, v);
        }
}
static void move_median_to_first(P* A, int64_t r, int64_t a, int64_t b, int64_t c) {
    if (comp(A[a], A[b])) {
        if (comp(A[b], A[c])) std::swap(A[r], A[b]);
        else if (comp(A[a], A[c])) std::swap(A[r], A[c]);
        else std::swap(A[r], A[a]);
    } else if (comp(A[a], A[c])) std::swap(A[r], A[a]);
    else if (comp(A[b], A[c])) std::swap(A[r], A[c]);
    else std::swap(A[r], A[b]);
}
static void insertion_sort(P* A, int64_t f, int64_t l) {
    if (f == l) return;
    for (int64_t i = f + 1; i != l; ++i) {
        P v = A[i];
        if (comp(v, A[f])) {
            for (int64_t j = i; j > f; --j) A[j] = A[j - 1];
            A[f] = v;
        } else {
            int64_t j = i;
            while (comp(v, A[j - 1])) { A[j] = A[j - 1]; --j; }
            A[j] = v;
        }
    }
}
static int lg(int64_t n) { int r = 0; while (n > 1) { n >>= 1; ++r; } return r; }

// data-parallel partition of [first+1, last) around pivot A[first]; returns the cut
static int64_t par_partition(P* A, int64_t first, int64_t last, std::vector<int64_t>& Lpos, std::vector<int64_t>& Rpos) {
    const uint32_t piv = K(A[first]);
    int64_t nL = 0, nR = 0;
    for (int64_t i = first; i < last; ++i) {             // one scan pass (prefix counts)
        if (i > first && K(A[i]) <= piv) Lpos[nL++] = i;  // left stop: !comp(A[i], pivot)
        if (K(A[i]) >= piv) Rpos[nR++] = i;               // right stop: !comp(pivot, A[i]) (pivot itself guards)
    }
    auto rr = [&](int64_t j) { return Rpos[nR - j]; };    // j-th right stop from the right (1-based)
    int64_t lo = 0, hi = std::min(nL, nR);                 // largest J with L_J < R_J (monotone)
    while (lo < hi) {
        int64_t mid = (lo + hi + 1) / 2;
        if (Lpos[mid - 1] < rr(mid)) lo = mid; else hi = mid - 1;
    }
    const int64_t J = lo;
    for (int64_t j = 1; j <= J; ++j) std::swap(A[Lpos[j - 1]], A[rr(j)]);
    int64_t cut = INT64_MAX;
    if (J < nL) cut = Lpos[J];
    if (J > 0) cut = std::min(cut, rr(J));
    return cut;
}

static void emul_nth(P* A, int64_t d, int64_t nth) {
    std::vector<int64_t> Lpos(d), Rpos(d);
    int64_t first = 0, last = d;
    int depth = lg(d) * 2;
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(A, first, nth + 1, last);
            std::swap(A[first], A[nth]);
            return;
        }
        --depth;
        const int64_t mid = first + (last - first) / 2;
        move_median_to_first(A, first, first + 1, mid, last - 1);
        const int64_t cut = par_partition(A, first, last, Lpos, Rpos);
        if (cut <= nth) first = cut; else last = cut;
    }
    insertion_sort(A, first, last);
}

int main() {
    std::mt19937_64 g(1);
    int bad = 0, tot = 0;
    for (int it = 0; it < 20000; ++it) {
        const int64_t d = 1 + g() % (it < 15000 ? 300 : 100000);
        const int distinct = 1 + g() % 6;
        std::vector<P> a(d);
        for (int64_t i = 0; i < d; ++i) {
            uint32_t key = (g() % 3 == 0) ? (uint32_t)(g() % 1000000) : (uint32_t)(g() % distinct);
            if (it % 7 == 0) key = (uint32_t)(i % distinct);                  // patterned
            if (it % 11 == 0) key = (uint32_t)(d - i) / (1 + distinct);       // sorted runs
            a[i] = ((P)key << 32) | (uint32_t)i;
        }
        const int64_t k = 1 + g() % d;
        std::vector<P> ref = a, emu = a;
        std::nth_element(ref.begin(), ref.begin() + (k - 1), ref.end(), comp);
        emul_nth(emu.data(), d, k - 1);
        ++tot;
        if (ref != emu) { if (bad < 5) printf("mismatch d=%ld k=%ld\n", (long)d, (long)k); ++bad; }
    }
    // heap path: partial_sort's heap_select
    for (int it = 0; it < 3000; ++it) {
        const int64_t d = 64 + g() % 50000;
        const int distinct = 1 + g() % 5;
        std::vector<P> a(d);
        for (int64_t i = 0; i < d; ++i) a[i] = ((P)(uint32_t)(g() % (g() % 2 ? distinct : 100000)) << 32) | (uint32_t)i;
        const int64_t k = 1 + g() % (d / 64);
        std::vector<P> ref = a, emu = a;
        std::partial_sort(ref.begin(), ref.begin() + k, ref.end(), comp);
        heap_select(emu.data(), 0, k, d);
        std::vector<P> s1(ref.begin(), ref.begin() + k), s2(emu.begin(), emu.begin() + k);
        std::sort(s1.begin(), s1.end()); std::sort(s2.begin(), s2.end());
        ++tot;
        if (s1 != s2) { if (bad < 10) printf("heap mismatch d=%ld k=%ld\n", (long)d, (long)k); ++bad; }
    }
    printf("cases %d mismatches %d\n", tot, bad);
    return bad != 0;
}
