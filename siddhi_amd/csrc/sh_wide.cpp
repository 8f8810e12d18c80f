// sh_wide.cpp — interning chains for group keys wider than one window key (sh_wide.h).
#include "sh_wide.h"

#include <cstring>
#include <string>

using namespace shd;

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t _e = (x);                                                           \
        if (_e != hipSuccess) return sh_fail(SH_ERR_DEVICE, hipGetErrorString(_e));    \
    } while (0)
#define RCHK(x)            \
    do {                   \
        int _r = (x);      \
        if (_r) return _r; \
    } while (0)

static bool wide64(int t) { return t == SH_T_LONG || t == SH_T_DOUBLE; }

bool WideKeys::needed(int n_group, const int32_t* group, const int32_t* types) {
    if (n_group > kKeyParts) return true;
    return n_group == 2 && (wide64(types[group[0]]) || wide64(types[group[1]]));
}

int WideKeys::init(int n_group, const int32_t* group, int n_cols, const int32_t* types, int64_t capacity) {
    if (n_group < 1 || n_group > SH_MAX_GROUP) return sh_fail(SH_ERR_INVALID, "bad group-by count");
    n = n_group;
    nl = 0;
    struct Comp { int src, out; };  // src >= 0 stream column, < 0 level id; out as WideLevel.out
    std::vector<Comp> comps;
    auto add_level = [&](int ncomp, const int* src, const int* srct, const int* out) {
        WideLevel& L = lv[nl];
        L = WideLevel{};
        L.kp.n = ncomp;
        for (int j = 0; j < ncomp; j++) {
            L.kp.col[j] = j;
            L.kp.type[j] = srct[j];
            L.src[j] = src[j];
            L.out[j] = out[j];
        }
        return nl++;
    };
    for (int i = 0; i < n; i++) {
        const int c = group[i];
        if (c < 0 || c >= n_cols) return sh_fail(SH_ERR_INVALID, "group-by column out of range");
        col[i] = c;
        type[i] = types[c];
        if (wide64(types[c])) {
            // its own level: the 64-bit value -> a 32-bit id
            const int src[1] = {c}, st[1] = {types[c]}, out[1] = {i};
            const int L = add_level(1, src, st, out);
            comps.push_back(Comp{-L - 1, -L - 1});
        } else {
            comps.push_back(Comp{c, i});
        }
    }
    auto comp_type = [&](const Comp& x) { return x.src >= 0 ? types[x.src] : (int)SH_T_STRID; };
    if (comps.size() >= 2) {
        int src[2] = {comps[0].src, comps[1].src}, st[2] = {comp_type(comps[0]), comp_type(comps[1])},
            out[2] = {comps[0].out, comps[1].out};
        int prev = add_level(2, src, st, out);
        for (size_t j = 2; j < comps.size(); j++) {
            int s2[2] = {-prev - 1, comps[j].src}, t2[2] = {SH_T_STRID, comp_type(comps[j])},
                o2[2] = {-prev - 1, comps[j].out};
            prev = add_level(2, s2, t2, o2);
        }
    } else if (comps[0].src >= 0) {
        // one 32-bit column (an aggregation pairs it with its bucket itself; interned only on request)
        const int src[1] = {comps[0].src}, st[1] = {types[comps[0].src]}, out[1] = {0};
        add_level(1, src, st, out);
    }
    for (int l = 0; l < nl; l++) RCHK(tab[l].init(std::max<int64_t>(capacity, 16)));
    return SH_OK;
}

WideDev WideKeys::dev() const {
    WideDev w{};
    w.nl = nl;
    w.last = nl - 1;
    for (int l = 0; l < nl; l++) {
        w.lv[l] = lv[l];
        w.lv[l].t = tab[l].dev();
    }
    return w;
}

int WideKeys::intern(hipStream_t s, const ColSet& full, const FilterProg& f, int64_t nev, const uint32_t** out) {
    *out = nullptr;
    for (int l = 0; l < nl; l++) RCHK(ids[l].reserve((size_t)std::max<int64_t>(nev, 1) * 4, false));
    const WideDev w = dev();
    for (int l = 0; l < nl; l++) {
        ColSet cs2{};
        cs2.n = w.lv[l].kp.n;
        const u32* prev = nullptr;
        bool first = true;
        for (int j = 0; j < cs2.n; j++) {
            const int src = w.lv[l].src[j];
            cs2.type[j] = w.lv[l].kp.type[j];
            if (src >= 0) {
                cs2.type[j] = full.type[src];  // (the column as loaded: a sharded owner's are 8-byte raw)
                cs2.ptr[j] = full.ptr[src];
            } else {
                cs2.ptr[j] = ids[-src - 1].p;
                prev = ids[-src - 1].as<u32>();  // (a level's id implies the event passed the filter)
                first = false;
            }
        }
        launch_wide_level(s, full, f, first ? 1 : 0, cs2, w.lv[l], prev, l == nl - 1 ? 1 : 0, nev, ids[l].as<u32>());
        HIPCHK(hipGetLastError());
    }
    for (int l = 0; l < nl; l++) RCHK(tab[l].check(s));
    *out = ids[nl - 1].as<uint32_t>();
    return SH_OK;
}

int WideKeys::decode(hipStream_t s, const int64_t* idv, int64_t nrows, int64_t* out) {
    if (nrows <= 0) return SH_OK;
    launch_wide_decode(s, dev(), idv, nrows, out);
    HIPCHK(hipGetLastError());
    return SH_OK;
}

int WideKeys::save(std::vector<uint8_t>& blob, hipStream_t s) {
    auto put = [&](int64_t v) { blob.insert(blob.end(), (const uint8_t*)&v, (const uint8_t*)&v + 8); };
    put(nl);
    for (int l = 0; l < nl; l++) {
        RCHK(tab[l].check(s));
        put(tab[l].n_keys);
        put((int64_t)tab[l].size_);
        const size_t o = blob.size(), bytes = tab[l].size_ * 8;
        blob.resize(o + bytes);
        HIPCHK(hipMemcpyAsync(blob.data() + o, tab[l].keys.p, bytes, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return SH_OK;
}

int WideKeys::load(const uint8_t* p, size_t len, size_t& off, hipStream_t s) {
    auto get = [&](int64_t& v) {
        if (off + 8 > len) return false;
        std::memcpy(&v, p + off, 8);
        off += 8;
        return true;
    };
    int64_t nl2 = 0;
    if (!get(nl2) || nl2 != nl) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated or of another group key");
    for (int l = 0; l < nl; l++) {
        int64_t nk = 0, size = 0;
        if (!get(nk) || !get(size) || size != (int64_t)tab[l].size_ || nk < 0 || nk > size + 1)
            return sh_fail(SH_ERR_INVALID, "snapshot blob truncated or of another group key");
        const size_t bytes = tab[l].size_ * 8;
        if (off + bytes > len) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        HIPCHK(hipMemcpyAsync(tab[l].keys.p, p + off, bytes, hipMemcpyHostToDevice, s));
        off += bytes;
        RCHK(tab[l].h_ctrl.reserve(16));
        uint32_t* c = tab[l].h_ctrl.as<uint32_t>();
        c[0] = (uint32_t)nk;
        c[1] = c[2] = c[3] = 0;
        HIPCHK(hipMemcpyAsync(tab[l].ctrl.p, c, 16, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        tab[l].n_keys = nk;
    }
    return SH_OK;
}
