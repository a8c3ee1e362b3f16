// Test helper: checks the host build of gf_orb_slam_amd/csrc/select.h (the
// libstdc++ introselect/heap port the device runs) against std::nth_element /
// std::priority_queue on random tie-heavy inputs.
#include <algorithm>
#include <cstdint>
#include <queue>
#include <random>
#include <vector>

#include "../../gf_orb_slam_amd/csrc/select.h"

extern "C" int select_check(int trials, int seed) {
    std::mt19937 rng(seed);
    for (int t = 0; t < trials; t++) {
        int n = 1 + rng() % 700;
        int range = 1 + rng() % 40;
        std::vector<uint32_t> a(n);
        for (int i = 0; i < n; i++) a[i] = ((uint32_t)(rng() % range) << 24) | (uint32_t)i;
        int k = rng() % n;
        std::vector<uint32_t> b = a;
        std::nth_element(b.begin(), b.begin() + k, b.end(),
                         [](uint32_t x, uint32_t y) { return (x >> 24) > (y >> 24); });
        gfsel::nth_element(a.data(), 0, k, n, gfsel::RespGreater());
        if (a != b) return -(t + 1);
        // heap: push all, pop all, compare order
        std::priority_queue<uint32_t, std::vector<uint32_t>, bool (*)(uint32_t, uint32_t)> pq(
            [](uint32_t x, uint32_t y) { return (x >> 24) < (y >> 24); });
        std::vector<uint32_t> h;
        auto lt = [](uint32_t x, uint32_t y) { return (x >> 24) < (y >> 24); };
        for (int i = 0; i < n; i++) {
            pq.push(b[i]);
            h.push_back(b[i]);
            gfsel::push_heap(h.data(), (int)h.size(), lt);
        }
        while (!pq.empty()) {
            if (pq.top() != h[0]) return -(100000 + t);
            pq.pop();
            gfsel::pop_heap(h.data(), (int)h.size(), lt);
            h.pop_back();
        }
    }
    return 0;
}
