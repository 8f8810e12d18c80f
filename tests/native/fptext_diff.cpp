// Differential check of the two restatements of Double.toString / Float.toString (the partition flow id of
// a double / float key): the oracle's jhm::fp_decimal (printf digit search) and the product's
// shj::java_fp_text (std::to_chars shortest form) over random bit patterns, decimal fractions and floats.
// Test code only.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "../../oracle/jhashmap.h"
#include "../../siddhi_amd/csrc/sh_jmap.h"

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 rng(7);
    long bad = 0;
    for (long i = 0; i < n; i++) {
        const uint64_t b = rng();
        const int mode = (int)(i % 4);
        double v;
        if (mode == 0) {
            std::memcpy(&v, &b, 8);
        } else if (mode == 1) {
            v = (double)(int64_t)(b % 2000001 - 1000000) / (double)(1 + (b >> 40) % 1000);
        } else if (mode == 2) {
            float f;
            const uint32_t w = (uint32_t)b;
            std::memcpy(&f, &w, 4);
            v = f;
        } else {
            v = (double)(float)((double)(int64_t)(b % 20001 - 10000) / (double)(1 + (b >> 40) % 100));
        }
        const bool f32 = mode >= 2;
        const std::u16string a = shj::java_fp_text(v, f32), c = jhm::fp_decimal(v, f32);
        if (a != c) {
            if (bad < 5) {
                std::string x(a.begin(), a.end()), y(c.begin(), c.end());
                printf("MISMATCH %s %.17g: product %s oracle %s\n", f32 ? "float" : "double", v, x.c_str(), y.c_str());
            }
            bad++;
        }
    }
    if (bad) return 1;
    printf("ok %ld values\n", n);
    return 0;
}
