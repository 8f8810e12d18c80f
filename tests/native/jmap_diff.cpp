// Differential check of the two independent restatements of java.util.HashMap<String, …> iteration
// order (JDK 8): the oracle's (oracle/jhashmap.h, pointer nodes mirroring HashMap / TreeNode) and the
// product's host scheduler (siddhi_amd/csrc/sh_jmap.h, pooled index nodes). Random computeIfAbsent /
// iterator-remove sequences over keys with heavy String.hashCode collisions ("Aa" == "BB" blocks), so
// bins turn into red-black trees, split on resize and fall back to lists. Test code only.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../oracle/jhashmap.h"
#include "../../siddhi_amd/csrc/sh_jmap.h"

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 200;
    std::vector<std::u16string> keys;
    std::vector<std::u16string> blocks = {u""};
    for (int i = 0; i < 5; i++) {  // 32 strings of one hash
        std::vector<std::u16string> nb;
        for (auto& b : blocks) { nb.push_back(b + u"Aa"); nb.push_back(b + u"BB"); }
        blocks.swap(nb);
    }
    for (auto& b : blocks) keys.push_back(b);
    for (auto& b : blocks) keys.push_back(b + u"x");  // another 32 of one hash
    for (int i = 0; i < 400; i++) {
        std::string s = std::to_string(i * 7919 % 100003);
        keys.push_back(std::u16string(s.begin(), s.end()));
    }
    long checks = 0, trees = 0;
    for (int r = 0; r < rounds; r++) {
        std::mt19937_64 rng(1000 + r);
        jhm::HashMap<int64_t> a;
        shj::JavaStringMap b;
        const int live_max = 20 + (int)(rng() % 300);
        std::vector<int> present(keys.size(), 0);
        int live = 0;
        for (int step = 0; step < 3000; step++) {
            const bool hot = rng() % 2;
            const size_t k = hot ? rng() % 64 : 64 + rng() % (keys.size() - 64);
            if (live < live_max && (rng() % 3 != 0 || !present[k])) {
                a.compute_if_absent(keys[k], (int64_t)k);
                b.touch(keys[k], (uint32_t)k);
                if (!present[k]) { present[k] = 1; live++; }
            } else {
                // remove a batch in iteration order, like returnAllStates
                std::vector<int64_t> order;
                a.for_each([&](const std::u16string&, int64_t v) { order.push_back(v); });
                for (int64_t v : order)
                    if (rng() % 4 == 0) {
                        a.remove(keys[(size_t)v]);
                        b.erase(keys[(size_t)v]);
                        present[(size_t)v] = 0;
                        live--;
                    }
            }
            std::vector<int64_t> oa, ob;
            a.for_each([&](const std::u16string&, int64_t v) { oa.push_back(v); });
            b.visit([&](uint32_t v) { ob.push_back(v); });
            checks++;
            if (oa.size() != (size_t)live || oa != std::vector<int64_t>(ob.begin(), ob.end())) {
                printf("MISMATCH round %d step %d live %d sizes %zu %zu\n", r, step, live, oa.size(), ob.size());
                return 1;
            }
            if (a.tree_bins() > 0) trees++;
        }
    }
    printf("ok %ld checks, %ld with tree bins\n", checks, trees);
    return trees > 0 ? 0 : 2;
}
