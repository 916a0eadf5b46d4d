// TEST INFRASTRUCTURE ONLY (oracle): torch.sort's CPU permutation for the top-p filter.
//
// The reference's top_k_top_p_filtering sorts a bf16 row with torch.sort(descending=True)
// (hf_export/modeling_t5gemma_voice.py:107-108). torch 2.10's CPU sort (stable=False) is
// libstdc++ std::sort over (value, index) pairs in index order with the value-only
// comparator `isnan(a) && !isnan(b) || a > b` (SURVEY a14' 5: 40/40 tie-laden probes and
// the reference-run sampler goldens agree). Compiled with g++ by __graft_entry__.build()
// into oracle/lib/liboracle_sort.so; tests compare the product's sparse emulation
// (csrc/sort_emu.h) with it.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

extern "C" void oracle_sort_desc(const float* v, int64_t n, int64_t* perm_out) {
    struct KV {
        float v;
        int64_t i;
    };
    std::vector<KV> a((size_t)n);
    for (int64_t i = 0; i < n; ++i) a[(size_t)i] = {v[i], i};
    std::sort(a.begin(), a.end(), [](const KV& x, const KV& y) {
        return (std::isnan(x.v) && !std::isnan(y.v)) || (x.v > y.v);
    });
    for (int64_t r = 0; r < n; ++r) perm_out[r] = a[(size_t)r].i;
}
