// CPU ORACLE (C++) — test infrastructure only, never the product path.
//
// Restatement of the reference's biased type quantizer (paths relative to the reference root):
//   NMSE_Results/Codes/All_Schemes.py:669-687  Type_biased_quantize
//   NMSE_Results/Codes/All_Schemes.py:644-666  Reznik
// with torch CPU semantics for every op whose float behaviour defines the output:
//   k' = floor(f32(m) * p + 0.5f)                                   (AS:648)
//   m' = k'.sum()   torch CPU cascade order (uqo_torch_sum)          (AS:649)
//   Delta = int(f32(m') - f32(m))                                    (AS:656)
//   topk: ATen TopKImpl.h on one slice — (value as double, index) pairs, comparator
//         "NaN first, then larger value"; std::partial_sort when k*64 <= n, else
//         std::nth_element (libstdc++, the library torch is built with); the selected
//         index SET is queue[0..k).                                  (AS:660, AS:664)
//   out = (L1 * sign(x)) * (k'/f32(m))                               (AS:687)
// `tie_mode` 0 reproduces torch's choice among equal values at the selection threshold;
// 1 takes the lowest indices among them (the GPU kernels' deterministic rule).
// Returns 0, or -1 (m' not finite: the reference raises ValueError) / -2 (|Delta| > d:
// torch.topk raises RuntimeError); `out` is then not written.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

extern "C" float uqo_torch_sum(const float* v, int64_t d, int torch_threads);
extern "C" float uqo_l1_torch_order(const float* x, int64_t d, int torch_threads, float* scratch);

namespace {
inline float torch_sign(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }
typedef std::pair<double, int64_t> elem_t;
inline bool nan_first_larger(const elem_t& x, const elem_t& y) {
    return (std::isnan(x.first) && !std::isnan(y.first)) || (x.first > y.first);
}
}  // namespace

extern "C" int uqo_biased_quantize(const float* x, float* out, int64_t d, int64_t m, int torch_threads,
                                   int tie_mode, float* l1_out, int64_t* delta_out, int32_t* ambiguous_out) {
    std::vector<float> scratch((size_t)std::max<int64_t>(d, 1));
    const float L = uqo_l1_torch_order(x, d, torch_threads, scratch.data());
    const float den = L + 1e-12f;
    const float fm = (float)m;
    std::vector<float> kp((size_t)d), mp((size_t)d);
    for (int64_t i = 0; i < d; ++i) {
        const float p = fabsf(x[i]) / den;         // AS:681 |x| / (L1 + 1e-12)
        mp[i] = fm * p;                            // m * p
        kp[i] = floorf(mp[i] + 0.5f);              // AS:648
    }
    const float mprime = uqo_torch_sum(kp.data(), d, torch_threads);   // AS:649
    int64_t Delta = 0;
    int32_t ambiguous = 0;
    if (!(mprime == fm)) {                          // AS:651
        if (!std::isfinite(mprime)) return -1;      // AS:656 int(nan/inf) raises
        Delta = (int64_t)(mprime - fm);             // AS:656 int() truncates toward zero
        const int64_t k = Delta > 0 ? Delta : -Delta;
        if (k > d) return -2;                       // AS:660/664 topk: k out of range
        if (k > 0) {
            std::vector<elem_t> q((size_t)d);
            for (int64_t i = 0; i < d; ++i) {
                const float dp = kp[i] - mp[i];                         // AS:655
                q[(size_t)i] = elem_t((double)(Delta > 0 ? dp : -dp), i);
            }
            std::vector<elem_t> sel;
            if (tie_mode == 0) {
                if (k * 64 <= d)
                    std::partial_sort(q.begin(), q.begin() + k, q.end(), nan_first_larger);
                else
                    std::nth_element(q.begin(), q.begin() + (k - 1), q.end(), nan_first_larger);
                sel.assign(q.begin(), q.begin() + k);
            } else {
                // stable: larger value first, ties by lower index
                std::vector<elem_t> s2 = q;
                std::stable_sort(s2.begin(), s2.end(), nan_first_larger);
                sel.assign(s2.begin(), s2.begin() + k);
            }
            // ambiguous = the threshold value also occurs outside the selected set
            const double thr = sel.back().first;
            int64_t in_sel = 0, total = 0;
            for (const auto& e : sel) in_sel += (e.first == thr);
            for (int64_t i = 0; i < d; ++i) total += (q[(size_t)i].first == thr);
            ambiguous = total > in_sel ? 1 : 0;
            for (const auto& e : sel) kp[(size_t)e.second] += Delta > 0 ? -1.f : 1.f;   // AS:661 / AS:665
        }
    }
    for (int64_t i = 0; i < d; ++i) out[i] = (L * torch_sign(x[i])) * (kp[i] / fm);   // AS:687
    if (l1_out) *l1_out = L;
    if (delta_out) *delta_out = Delta;
    if (ambiguous_out) *ambiguous_out = ambiguous;
    return 0;
}
