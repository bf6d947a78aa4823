// uq_legacy_rng.cpp — the NMSE drivers' input vectors, bit-identical to numpy's
// legacy RandomState and multi-threaded.  Host-only C++ (g++), linked into libuq_dme.so.
//
// What it replaces (ND = NMSE_Results/Codes/Normal_dist.py):
//   ND:14, 88-91   np.random.seed(42); per instance, n successive np.random.normal(0, 1, size=d)
//   Laplace_dist.py:89    np.random.laplace(loc=1, scale=2, size=d)
//   Gamma_dist.py:86      np.random.gamma(shape=2, scale=2, size=d)
//   Bernoulli_dist.py:90  np.random.choice(np.arange(2), size=d, p=[0.3, 0.7])
//   Lognormal_dist.py:90  np.random.lognormal(mean=1, sigma=2, size=d)
// The legacy samplers read one MT19937 word stream in order; n successive size-d calls are one
// size-n*d call (the gauss cache carries over, as in RandomState).  Per value (numpy's legacy
// distributions, restated; the CPU tests pin every one against RandomState itself):
//   next_double  = ((w0 >> 5) * 2^26 + (w1 >> 6)) / 2^53                       (2 words)
//   gauss        : the cached value if any, else polar attempts of 2 doubles
//                  x = 2u - 1 until 0 < r2 = x1*x1 + x2*x2 < 1; f = sqrt(-2 log(r2) / r2);
//                  cache f*x1, return f*x2
//   normal       = loc + scale * gauss             lognormal = exp(mean + sigma * gauss)
//   laplace      : u = next_double; u >= 0.5: loc - scale*log(2 - u - u); u > 0: loc + scale*log(u + u);
//                  u == 0: draw again
//   gamma (k > 1): Marsaglia-Tsang on gauss + next_double (b = k - 1/3, c = 1/sqrt(9b))
//   choice(p)    : u = next_double (random_sample), index = #{cdf <= u} (searchsorted 'right')
//   uniform      = low + range * next_double
// log / exp / sqrt are the host libm's, the same functions numpy calls, so the bits agree on the
// machine they run on (glibc picks its log variant per CPU; so does numpy's).  Built with
// -ffp-contract=off: every product and sum is rounded on its own, as numpy's baseline build does.
//
// Parallel form (speculative parsing).  The stream of words is cut into chunks; chunk k parses
// from its first word with an empty gauss cache, as if a value started there.  A sampler's state
// between values is (word position, has_gauss, gauss), and the next values depend on nothing
// else, so as soon as the true parse -- chunk k - 1's, run past its end -- reaches a state that
// chunk k's parse also passed through, chunk k's values from there on are the true ones.  For
// the fixed-stride samplers and for gauss (whose attempts all start 4 words apart) that happens
// at the first value; gamma's mixed draws meet within a few values.  If two chunks never meet
// within the overlap window, the wave ends at the first chunk's end and the next wave restarts
// from its (true) end state: slower, never wrong.  Chunk k reaches its start word by MT19937
// jump-ahead (uq_mt_poly.cpp).  ||v||^2 per vector is summed in f64 in a fixed order of the
// vector's own elements (not numpy's BLAS order, which depends on its thread count), then
// rounded through sqrt and squared as np.linalg.norm(v) ** 2 does.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <sys/mman.h>
#include <unistd.h>
#include <thread>
#include <vector>

extern "C" int uq_mt_jump_host(const uint32_t* state624, int64_t blocks, uint32_t* out624);

namespace {

constexpr int kN = 624;
constexpr int64_t kCkpt = 4096;          // a parse state every kCkpt values (for the exact end state)
// words a chunk parses past its end to meet the next chunk; words per chunk, at least (test hook:
// uq_legacy_test_params shrinks both to exercise many chunk boundaries and missed meetings)
std::atomic<int64_t> g_overlap{1 << 14};
std::atomic<int64_t> g_min_chunk{1 << 21};
std::atomic<int64_t> g_waves{0}, g_misses{0};
constexpr int64_t kNormBlock = 1 << 16;  // values per norm partial

enum Dist : int32_t { kNormal = 0, kLaplace = 1, kGamma = 2, kChoice2 = 3, kLognormal = 4, kUniform = 5 };

inline uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

inline void twist(uint32_t* s) {          // one MT19937 block, in place (numpy's mt19937_gen)
    int i = 0;
    for (; i < kN - 397; ++i) {
        const uint32_t y = (s[i] & 0x80000000u) | (s[i + 1] & 0x7fffffffu);
        s[i] = s[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    for (; i < kN - 1; ++i) {
        const uint32_t y = (s[i] & 0x80000000u) | (s[i + 1] & 0x7fffffffu);
        s[i] = s[i + 397 - kN] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    const uint32_t y = (s[kN - 1] & 0x80000000u) | (s[0] & 0x7fffffffu);
    s[kN - 1] = s[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

// The word stream of a RandomState whose key is `key` (block 0): absolute word a is word a % 624
// of block a / 624 (block b = b twists of block 0).  A RandomState at pos p reads word p next.
struct Stream {
    uint32_t s[kN];
    uint32_t t[kN];                       // s tempered (the words as drawn)
    int64_t blk = 0;
    int idx = 0;

    void temper_all() {
        for (int i = 0; i < kN; ++i) t[i] = temper(s[i]);
    }
    bool seek(const uint32_t* key, int64_t a) {
        blk = a / kN;
        idx = (int)(a % kN);
        std::memcpy(s, key, sizeof(s));
        if (blk <= 64) {
            for (int64_t b = 0; b < blk; ++b) twist(s);
        } else {
            uint32_t out[kN];
            if (uq_mt_jump_host(key, blk, out)) return false;
            std::memcpy(s, out, sizeof(s));
        }
        temper_all();
        return true;
    }
    int64_t pos() const { return blk * kN + idx; }
    inline uint32_t next() {
        if (idx == kN) {
            twist(s);
            temper_all();
            ++blk;
            idx = 0;
        }
        return t[idx++];
    }
    inline double next_double() {
        const int32_t a = (int32_t)(next() >> 5), b = (int32_t)(next() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
};

// Value buffers come from a process-wide pool: a C4 call draws ~3.4 GB of f64 values, and
// fresh pages for them every call (mmap'd, first-touch faults from every thread) cost more than
// the draws on a VM host.  New buffers are 2 MB aligned and advised as huge pages; returned ones
// are kept up to a quarter of physical memory (at most 32 GB).
class Pool {
  public:
    static Pool& get() {
        static Pool p;
        return p;
    }
    double* take(size_t& cap) {                         // at least cap doubles; cap := the real size
        {
            std::lock_guard<std::mutex> g(mu_);
            auto it = free_.lower_bound(cap);
            if (it != free_.end()) {
                cap = it->first;
                double* b = it->second;
                held_ -= it->first * sizeof(double);
                free_.erase(it);
                return b;
            }
        }
        const size_t bytes = ((cap * sizeof(double) + kAlign - 1) / kAlign) * kAlign;
        void* m = nullptr;
        if (posix_memalign(&m, kAlign, bytes)) return nullptr;
        madvise(m, bytes, MADV_HUGEPAGE);
        cap = bytes / sizeof(double);
        return static_cast<double*>(m);
    }
    void give(double* b, size_t cap) {
        if (!b) return;
        std::lock_guard<std::mutex> g(mu_);
        if (held_ + cap * sizeof(double) > limit_) {
            std::free(b);
            return;
        }
        held_ += cap * sizeof(double);
        free_.emplace(cap, b);
    }

  private:
    Pool() {
        const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
        const double phys = pages > 0 && psz > 0 ? (double)pages * (double)psz : 16e9;
        limit_ = (size_t)std::min(32e9, phys / 4);
    }
    static constexpr size_t kAlign = 2u << 20;
    std::mutex mu_;
    std::multimap<size_t, double*> free_;
    size_t held_ = 0, limit_ = 0;
};

// A growable array of doubles that does not initialise what it allocates.
struct DBuf {
    double* p = nullptr;
    size_t n = 0, cap = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
    DBuf& operator=(DBuf&& o) noexcept {
        if (this != &o) {
            Pool::get().give(p, cap);
            p = o.p; n = o.n; cap = o.cap;
            o.p = nullptr; o.n = o.cap = 0;
        }
        return *this;
    }
    ~DBuf() { Pool::get().give(p, cap); }
    void reserve(size_t c) {
        if (c <= cap) return;
        size_t nc = c;
        double* q = Pool::get().take(nc);
        if (!q) throw std::bad_alloc();
        if (n) std::memcpy(q, p, n * sizeof(double));
        Pool::get().give(p, cap);
        p = q;
        cap = nc;
    }
    void push_back(double v) {
        if (n == cap) reserve(cap ? 2 * cap : 1024);
        p[n++] = v;
    }
    double* data() { return p; }
    const double* data() const { return p; }
    size_t size() const { return n; }
};

struct PState {
    int64_t p;        // absolute index of the next word
    int32_t h;        // has_gauss
    double g;         // gauss (0.0 when h == 0, as numpy leaves it)
};

struct Par {
    double a, b;      // normal/lognormal: loc, scale; laplace: loc, scale; gamma: shape, scale;
                      // choice2: cdf[0], cdf[1]; uniform: low, range
    double gb, gc;    // gamma: b = shape - 1/3, c = 1/sqrt(9 b)
};

inline double gauss(Stream& w, int32_t& h, double& g) {
    if (h) {
        const double t = g;
        h = 0;
        g = 0.0;
        return t;
    }
    double x1, x2, r2;
    do {
        x1 = 2.0 * w.next_double() - 1.0;
        x2 = 2.0 * w.next_double() - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    g = f * x1;
    h = 1;
    return f * x2;
}

template <int D>
inline double draw(Stream& w, int32_t& h, double& g, const Par& q) {
    if constexpr (D == kNormal) {
        return q.a + q.b * gauss(w, h, g);
    } else if constexpr (D == kLognormal) {
        return std::exp(q.a + q.b * gauss(w, h, g));
    } else if constexpr (D == kLaplace) {
        for (;;) {
            const double u = w.next_double();
            if (u >= 0.5) return q.a - q.b * std::log(2.0 - u - u);
            if (u > 0.0) return q.a + q.b * std::log(u + u);
        }
    } else if constexpr (D == kGamma) {
        for (;;) {
            double X, V;
            do {
                X = gauss(w, h, g);
                V = 1.0 + q.gc * X;
            } while (V <= 0.0);
            V = V * V * V;
            const double U = w.next_double();
            if (U < 1.0 - 0.0331 * (X * X) * (X * X)) return q.b * (q.gb * V);
            if (std::log(U) < 0.5 * X * X + q.gb * (1. - V + std::log(V))) return q.b * (q.gb * V);
        }
    } else if constexpr (D == kChoice2) {
        const double u = w.next_double();
        return (double)((q.a <= u) + (q.b <= u));
    } else {
        return q.a + q.b * w.next_double();
    }
}

constexpr bool uses_gauss(int d) { return d == kNormal || d == kLognormal || d == kGamma; }

inline bool same_state(const PState& x, const PState& y, bool ug) {
    if (x.p != y.p) return false;
    if (!ug) return true;
    if (x.h != y.h) return false;
    return !x.h || std::memcmp(&x.g, &y.g, sizeof(double)) == 0;
}

double words_per_value(int d) {
    switch (d) {
        case kNormal:
        case kLognormal: return 2.0 / 0.7853981633974483;   // 4 words per attempt, 2 values per accept
        case kGamma: return 4.75;
        default: return 2.0;
    }
}

struct JState {
    int64_t j;                      // value index within the chunk's parse
    PState st;                      // the state before value j
};

struct Chunk {
    int64_t w0 = 0, w1 = 0, stop = 0;
    PState start{};
    DBuf vals;
    std::vector<PState> head;       // state before value j, j = 0.., while p < w0 + overlap
    std::vector<JState> tail;       // states with p >= w1, in order
    std::vector<JState> ckpt;       // every kCkpt-th state, in order
    PState end{};
    bool ok = true;
    // gamma: the parse from w0 + 2 (the other phase, see parse_chunk); it merges into this one
    // at (alt_j, pri_j) when both reach the same state, and is materialised only if chosen
    std::vector<Chunk> alt;
    bool merged = false;
    int64_t alt_j = 0, pri_j = 0;
};

template <int D>
struct Parser {
    Stream w;
    int32_t h = 0;
    double g = 0.0;
    PState st{};
    int64_t j = 0, head_end = 0;
    Chunk* c = nullptr;
    bool rec_head = false;

    bool init(const uint32_t* key, Chunk* ch, PState start, bool record_head) {
        c = ch;
        rec_head = record_head;
        head_end = ch->w0 + g_overlap.load();
        if (!w.seek(key, start.p)) return false;
        h = start.h;
        g = start.g;
        st = start;
        c->vals.reserve((size_t)((double)(c->stop - c->w0) / words_per_value(D) * 1.02) + 64);
        record();
        return true;
    }
    void record() {
        if (rec_head && st.p < head_end) c->head.push_back(st);
        if (st.p >= c->w1) c->tail.push_back(JState{j, st});
        if (j % kCkpt == 0) c->ckpt.push_back(JState{j, st});
    }
    void step(const Par& q) {
        c->vals.push_back(draw<D>(w, h, g, q));
        st = PState{w.pos(), h, g};
        ++j;
        record();
    }
    // The same steps while st.p < limit (<= c->w1), for a parse past its head window: locals in
    // registers, checkpoints only at their boundaries; a state reaching w1 is recorded as tail.
    void run_body(const Par& q, int64_t limit) {
        if (st.p >= limit) return;
        int32_t hh = h;
        double gg = g;
        int64_t jj = j, p = st.p;
        DBuf& V = c->vals;
        const double wpv = words_per_value(D);
        while (p < limit) {
            const int64_t cnt = (jj / kCkpt + 1) * kCkpt - jj;
            if (V.cap < V.n + (size_t)cnt)
                V.reserve(std::max(V.n + (size_t)cnt, V.n + (size_t)((double)(limit - p) / wpv * 1.02) + 64));
            double* o = V.data() + V.n;
            int64_t k = 0;
            for (; k < cnt && p < limit; ++k) {
                o[k] = draw<D>(w, hh, gg, q);
                p = w.pos();
            }
            V.n += (size_t)k;
            jj += k;
            if (jj % kCkpt == 0) c->ckpt.push_back(JState{jj, PState{p, hh, gg}});
        }
        h = hh;
        g = gg;
        j = jj;
        st = PState{p, hh, gg};
        if (st.p >= c->w1) c->tail.push_back(JState{j, st});
    }
};

// Gamma's phase: with p the word position and h the cache flag, (p / 2 + h) mod 2 is kept by
// every value (an X flips it, its U flips it back) and changes only when V = 1 + cX <= 0 rejects
// an X (X < -3.87, about 5e-5 of them).  A parse started in the other phase than the true one
// would not meet it for ~10^4 values, so a gamma chunk also parses from w0 + 2 (the other phase)
// in lockstep with the primary parse until the two meet -- typically after the next such
// rejection, a few percent of the chunk -- and the stitch takes whichever meets the true parse.
template <int D>
void parse_chunk(const uint32_t* key, const Par& q, Chunk& c, bool speculative) {
    Parser<D> A;
    if (!A.init(key, &c, c.start, speculative)) {
        c.ok = false;
        return;
    }
    auto finish = [&]() {                    // A from here to its stop
        if (speculative)
            while (A.st.p < A.head_end && A.st.p < c.stop) A.step(q);
        A.run_body(q, std::min(c.w1, c.stop));
        while (A.st.p < c.stop) A.step(q);
        c.end = A.st;
    };
    if (D != kGamma || !speculative) {
        finish();
        return;
    }
    c.alt.resize(1);
    Chunk& b = c.alt[0];
    b.w0 = c.w0;
    b.w1 = c.w1;
    b.stop = c.stop;
    b.start = PState{c.w0 + 2, 0, 0.0};
    Parser<D> B;
    if (!B.init(key, &b, b.start, true)) {
        c.ok = false;
        return;
    }
    for (;;) {
        if (A.st.p == B.st.p && same_state(A.st, B.st, true)) {
            c.merged = true;
            c.alt_j = B.j;
            c.pri_j = A.j;
            break;
        }
        const bool a_live = A.st.p < c.stop, b_live = B.st.p < c.stop;
        if (b_live && (!a_live || B.st.p <= A.st.p)) B.step(q);
        else if (a_live) A.step(q);
        else break;
    }
    b.end = B.st;
    finish();
}

// Chunk c's alternative parse as the chunk itself (merged: its prefix, then the primary's rest).
void take_alt(Chunk& c) {
    Chunk& b = c.alt[0];
    if (c.merged) {
        const int64_t shift = c.alt_j - c.pri_j;
        b.vals.n = (size_t)c.alt_j;
        const size_t rest = c.vals.size() - (size_t)c.pri_j;
        b.vals.reserve(b.vals.n + rest);
        if (rest) std::memcpy(b.vals.data() + b.vals.n, c.vals.data() + c.pri_j, rest * sizeof(double));
        b.vals.n += rest;
        auto cut = [](std::vector<JState>& v, int64_t j) {
            v.erase(std::remove_if(v.begin(), v.end(), [j](const JState& x) { return x.j > j; }), v.end());
        };
        cut(b.tail, c.alt_j);
        cut(b.ckpt, c.alt_j);
        for (const JState& x : c.tail)
            if (x.j > c.pri_j) b.tail.push_back(JState{x.j + shift, x.st});
        for (const JState& x : c.ckpt)
            if (x.j > c.pri_j) b.ckpt.push_back(JState{x.j + shift, x.st});
        b.end = c.end;
    }
    std::swap(c.vals, b.vals);
    c.head.swap(b.head);
    c.tail.swap(b.tail);
    c.ckpt.swap(b.ckpt);
    c.end = b.end;
    c.start = b.start;
    c.alt.clear();
    c.merged = false;
}

template <class F>
void parallel_for(int threads, int64_t ntasks, F&& fn) {
    if (threads <= 1 || ntasks <= 1) {
        for (int64_t t = 0; t < ntasks; ++t) fn(t);
        return;
    }
    std::atomic<int64_t> nxt{0};
    auto body = [&]() {
        for (int64_t t; (t = nxt.fetch_add(1)) < ntasks;) fn(t);
    };
    const int nt = (int)std::min<int64_t>(threads, ntasks);
    std::vector<std::thread> pool;
    pool.reserve(nt - 1);
    for (int i = 1; i < nt; ++i) pool.emplace_back(body);
    body();
    for (auto& th : pool) th.join();
}

struct Segment {
    int64_t g0;                     // global value index of the first value
    const double* v;
    int64_t len;
};

// The state of a parse after `count` values from `from` (sequential).
template <int D>
bool advance(const uint32_t* key, const Par& q, PState from, int64_t count, PState* out) {
    Stream w;
    if (!w.seek(key, from.p)) return false;
    int32_t h = from.h;
    double g = from.g;
    for (int64_t j = 0; j < count; ++j) (void)draw<D>(w, h, g, q);
    *out = PState{w.pos(), h, g};
    return true;
}

// Where the true parse, at tail state x of chunk c, meets chunk nx: (which parse, head index).
int64_t find_head(const Chunk& nx, const PState& x, bool ug) {
    auto it = std::lower_bound(nx.head.begin(), nx.head.end(), x.p, [](const PState& a, int64_t p) { return a.p < p; });
    for (; it != nx.head.end() && it->p == x.p; ++it)
        if (same_state(*it, x, ug)) return it - nx.head.begin();
    return -1;
}

template <int D>
int draw_all(uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss_v, const Par& q, int64_t n, int64_t d,
             float* out, double* norm2, int threads) {
    const auto t_start = std::chrono::steady_clock::now();
    const bool ug = uses_gauss(D);
    const int64_t total = n * d;
    PState cur{(int64_t)*pos, ug ? *has_gauss : 0, ug ? *gauss_v : 0.0};
    std::vector<std::vector<Chunk>> waves;   // every chunk kept until the scatter (its values)
    std::vector<Segment> segs;
    int64_t have = 0;
    double wpv = words_per_value(D);
    while (have < total) {
        const int64_t need = total - have;
        const int64_t words = (int64_t)((double)need * wpv * 1.01) + 65536;
        const int64_t overlap = g_overlap.load(), min_chunk = std::max<int64_t>(g_min_chunk.load(), 2 * overlap);
        int64_t K = std::max<int64_t>(1, std::min<int64_t>((int64_t)threads * 4, words / min_chunk));
        if (threads <= 1) K = 1;
        // a multiple of 4 words: gauss attempts (4 words) of every chunk then sit on the true
        // parse's attempt grid, and every other draw is 2 words
        const int64_t csz = ((words + K - 1) / K + 3) & ~(int64_t)3;
        g_waves.fetch_add(1);
        waves.emplace_back((size_t)K);
        std::vector<Chunk>& ch = waves.back();
        for (int64_t k = 0; k < K; ++k) {
            Chunk& c = ch[(size_t)k];
            c.w0 = cur.p + k * csz;
            c.w1 = c.w0 + csz;
            c.stop = k + 1 < K ? c.w1 + overlap : c.w1;
            c.start = k ? PState{c.w0, 0, 0.0} : cur;
        }
        parallel_for(threads, K, [&](int64_t k) { parse_chunk<D>(key, q, ch[(size_t)k], k > 0); });
        for (int64_t k = 0; k < K; ++k)
            if (!ch[(size_t)k].ok) return -2;
        // stitch: chunk k's values [s, e) are the true ones
        int64_t s = 0;
        PState wave_end = cur;
        int64_t wave_vals = 0;
        for (int64_t k = 0; k < K; ++k) {
            Chunk& c = ch[(size_t)k];
            int64_t e = (int64_t)c.vals.size();
            int64_t s_next = -1;
            bool next_alt = false;
            if (k + 1 < K) {
                const Chunk& nx = ch[(size_t)k + 1];
                for (size_t t = 0; t < c.tail.size() && s_next < 0; ++t) {
                    const JState& x = c.tail[t];
                    if (x.j < s) continue;
                    int64_t hi = find_head(nx, x.st, ug);
                    if (hi < 0 && !nx.alt.empty()) {
                        hi = find_head(nx.alt[0], x.st, ug);
                        next_alt = hi >= 0;
                    }
                    if (hi >= 0) {
                        e = x.j;
                        s_next = hi;
                    }
                }
            }
            if (e < s) e = s;
            const int64_t take = std::min<int64_t>(e - s, need - wave_vals);
            if (take > 0) segs.push_back(Segment{have + wave_vals, c.vals.data() + s, take});
            if (wave_vals + take >= need) {     // done inside this chunk: the state after value s + take
                const int64_t j = s + take;
                PState from = k ? c.head[(size_t)s] : cur;
                int64_t fj = s;
                if (k == 0 && s != 0) return -3;
                for (const JState& x : c.ckpt)
                    if (x.j >= s && x.j <= j && x.j > fj) {
                        from = x.st;
                        fj = x.j;
                    }
                if (!advance<D>(key, q, from, j - fj, &wave_end)) return -2;
                wave_vals += take;
                break;
            }
            wave_vals += take;
            if (s_next < 0) {                    // last chunk, or no meeting: the wave ends here
                if (k + 1 < K) g_misses.fetch_add(1);
                wave_end = c.end;
                break;
            }
            if (next_alt) take_alt(ch[(size_t)k + 1]);
            s = s_next;
        }
        for (Chunk& c : ch) c.alt.clear();   // alternatives not taken
        have += wave_vals;
        if (have < total && wave_vals == 0 && wave_end.p == cur.p) return -3;   // no progress (cannot happen)
        if (wave_vals > 0) wpv = std::max(1.0, (double)(wave_end.p - cur.p) / (double)wave_vals);
        cur = wave_end;
    }
    const auto t_scatter = std::chrono::steady_clock::now();
    // scatter: f32 values and ||v||^2 of each vector, in a fixed order of the vector's elements
    const int64_t nb = (d + kNormBlock - 1) / kNormBlock;
    std::vector<double> part((size_t)(n * nb), 0.0);
    parallel_for(threads, n * nb, [&](int64_t t) {
        const int64_t i = t / nb, b = t % nb;
        int64_t g0 = i * d + b * kNormBlock;
        const int64_t g1 = std::min(i * d + d, g0 + kNormBlock);
        auto it = std::upper_bound(segs.begin(), segs.end(), g0, [](int64_t g, const Segment& sg) { return g < sg.g0; });
        size_t si = (size_t)(it - segs.begin()) - 1;
        double acc[4] = {0.0, 0.0, 0.0, 0.0};   // element e of the block -> acc[e % 4]
        int64_t lane = 0;
        while (g0 < g1) {
            const Segment& sg = segs[si];
            const int64_t off = g0 - sg.g0;
            const int64_t m = std::min(g1 - g0, sg.len - off);
            const double* v = sg.v + off;
            float* o = out + g0;
            for (int64_t k = 0; k < m; ++k) {
                const double x = v[k];
                o[k] = (float)x;
                acc[(lane + k) & 3] += x * x;
            }
            lane += m;
            g0 += m;
            ++si;
        }
        part[(size_t)t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    });
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t b = 0; b < nb; ++b) s += part[(size_t)(i * nb + b)];
        const double r = std::sqrt(s);
        norm2[i] = r * r;                       // np.linalg.norm(v) ** 2
    }
    if (std::getenv("UQDME_LEGACY_PROF"))
        std::fprintf(stderr, "legacy_draw: parse %.1f ms, scatter %.1f ms\n",
                     std::chrono::duration<double, std::milli>(t_scatter - t_start).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_scatter).count());
    // the RandomState after the draws: key = the block holding word cur.p - 1, pos = its index + 1
    if (cur.p != (int64_t)*pos) {
        const int64_t last = cur.p - 1;
        Stream w;
        if (!w.seek(key, (last / kN) * kN)) return -2;
        std::memcpy(key, w.s, sizeof(w.s));
        *pos = (int32_t)(last % kN) + 1;
    }
    if (ug) {
        *has_gauss = cur.h;
        *gauss_v = cur.g;
    }
    return 0;
}

}  // namespace

// n successive RandomState.<dist>(size=d) draws of the legacy state (key, pos, has_gauss, gauss)
// -- numpy's get_state() tuple -- into out [n][d] as f32 (the drivers' torch.as_tensor(..., f32)),
// with norm2[i] = np.linalg.norm(v_i) ** 2 (to f64 rounding, see above); the state is advanced in
// place.  dist: 0 normal(a = loc, b = scale), 1 laplace(loc, scale), 2 gamma(shape > 1, scale),
// 3 choice(arange(2), p) with a, b = the normalised cdf, 4 lognormal(mean, sigma),
// 5 uniform(a = low, b = high - low).  Returns 0, -1 on bad arguments, -2 if the jump-ahead is
// unavailable, -3 on an internal inconsistency.
extern "C" int uq_legacy_draw_f32(uint32_t* key624, int32_t* pos, int32_t* has_gauss, double* gauss_v,
                                  int32_t dist, double a, double b, int64_t n, int64_t d, float* out,
                                  double* norm2, int32_t threads) {
    if (!key624 || !pos || !has_gauss || !gauss_v || n < 0 || d < 0) return -1;
    if (*pos < 0 || *pos > kN) return -1;
    if (n == 0) return 0;
    if (d == 0) {
        if (norm2)
            for (int64_t i = 0; i < n; ++i) norm2[i] = 0.0;
        return norm2 ? 0 : -1;
    }
    if (!out || !norm2) return -1;
    if (n > ((int64_t)1 << 40) / d) return -1;
    Par q{a, b, 0.0, 0.0};
    if (dist == kGamma) {
        if (!(a > 1.0)) return -1;           // only the shape > 1 branch (the drivers' shape = 2)
        q.gb = a - 1. / 3.;
        q.gc = 1. / std::sqrt(9 * q.gb);
    }
    const int th = std::max(1, std::min<int32_t>(threads, 256));
    switch (dist) {
        case kNormal: return draw_all<kNormal>(key624, pos, has_gauss, gauss_v, q, n, d, out, norm2, th);
        case kLaplace: return draw_all<kLaplace>(key624, pos, has_gauss, gauss_v, q, n, d, out, norm2, th);
        case kGamma: return draw_all<kGamma>(key624, pos, has_gauss, gauss_v, q, n, d, out, norm2, th);
        case kChoice2: return draw_all<kChoice2>(key624, pos, has_gauss, gauss_v, q, n, d, out, norm2, th);
        case kLognormal: return draw_all<kLognormal>(key624, pos, has_gauss, gauss_v, q, n, d, out, norm2, th);
        case kUniform: return draw_all<kUniform>(key624, pos, has_gauss, gauss_v, q, n, d, out, norm2, th);
        default: return -1;
    }
}

// Test hook: set the chunking (values > 0; 0 keeps the current one) and read the counters of
// waves and missed chunk meetings since the last call (which resets them).
extern "C" int uq_legacy_test_params(int64_t min_chunk, int64_t overlap, int64_t* waves, int64_t* misses) {
    if (min_chunk < 0 || overlap < 0) return -1;
    if (min_chunk) g_min_chunk.store(min_chunk);
    if (overlap) g_overlap.store(overlap);
    if (waves) *waves = g_waves.exchange(0);
    if (misses) *misses = g_misses.exchange(0);
    return 0;
}
