// sh_jmap.h — iteration order of java.util.HashMap<String, …> (JDK 8, the reference's target:
// pom.xml:809), host side of the partitioned Scheduler (sh_plane.cpp).
//
// Scheduler.onTimeChange (core/util/Scheduler.java:71-104) walks PartitionStateHolder.states — a
// HashMap<String, Map<String, State>> keyed by String.valueOf(partition key) (PartitionStateHolder.java:36,
// 46; ValuePartitionExecutor.java:34-40) — and keeps, per distinct due time, only the first due state it
// meets (TreeMultimap values comparing equal, Scheduler.java:363-366). The map holds exactly the
// partitions whose notify queue is non-empty: notifyAt inserts through computeIfAbsent, returnAllStates
// removes emptied states through the iterator (PartitionStateHolder.java:132-161). The order therefore
// depends on the hash of each key and the history of the table; this class keeps that history:
//   * computeIfAbsent: resize first when size > threshold (even for a present key); new keys go to the
//     head of their bin; a bin that already had >= 7 nodes becomes a red-black tree (or the table doubles
//     while shorter than 64);
//   * resize: capacity 16 doubling at 0.75 load, never shrinking; bins split into lo / hi halves in order
//     (tree halves of <= 6 nodes become lists, others are rebuilt as trees);
//   * tree bins order their nodes by (spread hash, String.compareTo); a new node is linked right after its
//     tree parent and the root is moved to the bin's front; iterator removal (movable = false) unlinks and
//     rebalances, turning a tree whose root lacks a child or left grandchild back into a list (JDK 8).
// Nodes are slots of a pool addressed by int32 (-1 = null); a node's payload is the partition's slot.
#pragma once
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace shj {

inline int32_t java_string_hash(const std::u16string& s) {
    uint32_t h = 0;
    for (char16_t c : s) h = h * 31u + c;
    return (int32_t)h;
}

// Double.toString / Float.toString (String.valueOf of a double / float partition key) per the published
// specification (java.lang.Double#toString(double), JDK 8 javadoc): the fewest significant digits that still
// single the value out among its type's values — at least two when one would do and a two-digit decimal
// rounding to the value is nearer to it (Double.MIN_VALUE is "4.9E-324") —, plain notation for
// 10^-3 <= |v| < 10^7 ("100.0", "0.001"), otherwise "d.dddE<n>". JDK 8's FloatingDecimal prints a few values
// with more digits than this (JDK-4511638, fixed in JDK 19); partition keys hitting those are not restated.
inline std::u16string java_fp_text(double v, bool f32) {
    if (v != v) return u"NaN";
    if (v == 0) return std::signbit(v) ? u"-0.0" : u"0.0";
    if (std::isinf(v)) return v > 0 ? u"Infinity" : u"-Infinity";
    char buf[64];
    auto sci = [&](int prec) -> std::string {  // shortest (prec < 0) or prec + 1 significant digits
        std::to_chars_result r = prec < 0 ? (f32 ? std::to_chars(buf, buf + 63, (float)v, std::chars_format::scientific)
                                                 : std::to_chars(buf, buf + 63, v, std::chars_format::scientific))
                                          : std::to_chars(buf, buf + 63, v, std::chars_format::scientific, prec);
        return std::string(buf, r.ptr);
    };
    auto rounds_to_v = [&](const std::string& s) {
        return f32 ? std::strtof(s.c_str(), nullptr) == (float)v : std::strtod(s.c_str(), nullptr) == v;
    };
    std::string s = sci(-1);
    std::string two = sci(1);
    // digits and decimal exponent of "-d.ddde±x"
    auto split = [](const std::string& t, std::string& dig, int& ex) {
        const size_t e = t.find('e');
        dig.clear();
        for (size_t i = 0; i < e; i++)
            if (t[i] >= '0' && t[i] <= '9') dig.push_back(t[i]);
        ex = std::atoi(t.c_str() + e + 1);
        while (dig.size() > 1 && dig.back() == '0') dig.pop_back();
    };
    std::string dig;
    int ex = 0;
    split(s, dig, ex);
    if (dig.size() == 1 && rounds_to_v(two)) {
        // (both texts read back as v: their distances to it are compared in long double)
        const long double lv = v;
        const long double a = std::fabs(std::strtold(s.c_str(), nullptr) - lv),
                          b = std::fabs(std::strtold(two.c_str(), nullptr) - lv);
        if (b < a) split(two, dig, ex);
    }
    std::string o = v < 0 ? "-" : "";
    const double m = std::fabs(v);
    if (m >= 1e-3 && m < 1e7) {
        if (ex >= 0) {
            for (int i = 0; i <= ex; i++) o.push_back(i < (int)dig.size() ? dig[i] : '0');
            o.push_back('.');
            o += (int)dig.size() > ex + 1 ? dig.substr(ex + 1) : "0";
        } else {
            o += "0.";
            o.append(-ex - 1, '0');
            o += dig;
        }
    } else {
        o.push_back(dig[0]);
        o.push_back('.');
        o += dig.size() > 1 ? dig.substr(1) : "0";
        o += "E" + std::to_string(ex);
    }
    return std::u16string(o.begin(), o.end());
}

class JavaStringMap {
   public:
    static constexpr int32_t NIL = -1;

    int32_t size() const { return count_; }

    // computeIfAbsent(key, …) with `slot` as the value of a new entry
    void touch(const std::u16string& key, uint32_t slot) {
        const int32_t h = java_string_hash(key) ^ (int32_t)((uint32_t)java_string_hash(key) >> 16);
        if (count_ > threshold_ || bins_.empty()) grow();
        const int32_t b = bin_of(h);
        const int32_t head = bins_[b];
        if (by_key_.count(key)) return;
        int32_t len = 0;
        bool is_tree = head != NIL && nd_[head].tree;
        if (!is_tree)
            for (int32_t e = head; e != NIL; e = nd_[e].next) ++len;
        const int32_t x = alloc(h, key, slot);
        if (is_tree) {
            tree_insert(head, x);
        } else {
            nd_[x].next = head;
            bins_[b] = x;
            if (len >= 7) make_tree_bin(h);
        }
        ++count_;
    }

    // HashIterator.remove of the entry `key`
    void erase(const std::u16string& key) {
        auto it = by_key_.find(key);
        if (it == by_key_.end()) return;
        const int32_t x = it->second;
        const int32_t b = bin_of(nd_[x].hash);
        if (nd_[x].tree) {
            tree_erase(x);
        } else if (bins_[b] == x) {
            bins_[b] = nd_[x].next;
        } else {
            int32_t p = bins_[b];
            while (nd_[p].next != x) p = nd_[p].next;
            nd_[p].next = nd_[x].next;
        }
        by_key_.erase(it);
        free_.push_back(x);
        --count_;
    }

    // (bin, position along the bin's links): the lexicographic order of ranks is the iteration order
    bool rank(const std::u16string& key, int64_t* r) const {
        auto it = by_key_.find(key);
        if (it == by_key_.end()) return false;
        const int32_t b = bin_of(nd_[it->second].hash);
        int64_t pos = 0;
        for (int32_t e = bins_[b]; e != it->second; e = nd_[e].next) ++pos;
        *r = ((int64_t)b << 32) | pos;
        return true;
    }

    // the whole table (nodes, links, free list), so a checkpoint restores the iteration order exactly
    void save(std::vector<uint8_t>& out) const {
        auto put = [&](const void* p, size_t n) { out.insert(out.end(), (const uint8_t*)p, (const uint8_t*)p + n); };
        const int32_t hdr[4] = {count_, threshold_, (int32_t)bins_.size(), (int32_t)nd_.size()};
        put(hdr, sizeof(hdr));
        put(bins_.data(), bins_.size() * 4);
        for (const N& z : nd_) {
            const int32_t w[7] = {z.hash, (int32_t)z.slot, z.next, z.prev, z.up, z.lo, z.hi};
            const uint8_t fl = (z.tree ? 1 : 0) | (z.red ? 2 : 0);
            const uint32_t len = (uint32_t)z.key.size();
            put(w, sizeof(w));
            put(&fl, 1);
            put(&len, 4);
            put(z.key.data(), len * 2);
        }
        const int32_t nf = (int32_t)free_.size();
        put(&nf, 4);
        put(free_.data(), free_.size() * 4);
    }

    bool load(const uint8_t* p, size_t n) {
        size_t o = 0;
        auto get = [&](void* d, size_t k) {
            if (o + k > n) return false;
            std::memcpy(d, p + o, k);
            o += k;
            return true;
        };
        int32_t hdr[4];
        if (!get(hdr, sizeof(hdr)) || hdr[2] < 0 || hdr[3] < 0 || (hdr[2] & (hdr[2] - 1))) return false;
        JavaStringMap m;
        m.count_ = hdr[0];
        m.threshold_ = hdr[1];
        m.bins_.resize((size_t)hdr[2]);
        if (!get(m.bins_.data(), m.bins_.size() * 4)) return false;
        m.nd_.resize((size_t)hdr[3]);
        for (N& z : m.nd_) {
            int32_t w[7];
            uint8_t fl;
            uint32_t len;
            if (!get(w, sizeof(w)) || !get(&fl, 1) || !get(&len, 4) || len > (1u << 24)) return false;
            z.hash = w[0]; z.slot = (uint32_t)w[1]; z.next = w[2]; z.prev = w[3]; z.up = w[4]; z.lo = w[5]; z.hi = w[6];
            z.tree = fl & 1;
            z.red = (fl & 2) != 0;
            z.key.resize(len);
            if (!get(&z.key[0], (size_t)len * 2)) return false;
        }
        int32_t nf;
        if (!get(&nf, 4) || nf < 0 || nf > hdr[3]) return false;
        m.free_.resize((size_t)nf);
        if (!get(m.free_.data(), m.free_.size() * 4)) return false;
        std::vector<char> is_free(m.nd_.size(), 0);
        for (int32_t f : m.free_) {
            if (f < 0 || f >= hdr[3]) return false;
            is_free[(size_t)f] = 1;
        }
        for (size_t i = 0; i < m.nd_.size(); i++)
            if (!is_free[i]) m.by_key_[m.nd_[i].key] = (int32_t)i;
        if ((int32_t)m.by_key_.size() != m.count_) return false;
        *this = std::move(m);
        return true;
    }

    template <class F>
    void visit_keys(F f) const {
        for (int32_t head : bins_)
            for (int32_t e = head; e != NIL; e = nd_[e].next) f(nd_[e].slot, nd_[e].key);
    }

    template <class F>
    void visit(F f) const {
        for (int32_t head : bins_)
            for (int32_t e = head; e != NIL; e = nd_[e].next) f(nd_[e].slot);
    }

   private:
    struct N {
        int32_t hash = 0;
        uint32_t slot = 0;
        int32_t next = NIL, prev = NIL, up = NIL, lo = NIL, hi = NIL;
        bool tree = false, red = false;
        std::u16string key;
    };
    std::vector<N> nd_;
    std::vector<int32_t> free_, bins_;
    std::unordered_map<std::u16string, int32_t> by_key_;
    int32_t count_ = 0, threshold_ = 0;

    int32_t bin_of(int32_t h) const { return h & (int32_t)(bins_.size() - 1); }

    int32_t alloc(int32_t h, const std::u16string& key, uint32_t slot) {
        int32_t x;
        if (!free_.empty()) { x = free_.back(); free_.pop_back(); nd_[x] = N(); }
        else { x = (int32_t)nd_.size(); nd_.emplace_back(); }
        nd_[x].hash = h;
        nd_[x].slot = slot;
        nd_[x].key = key;
        by_key_[key] = x;
        return x;
    }

    // before: a (hash, key) b? (signed hash compare, then UTF-16 code unit order; keys are distinct)
    bool goes_left(int32_t x, int32_t p) const {
        if (nd_[p].hash != nd_[x].hash) return nd_[p].hash > nd_[x].hash;
        return nd_[x].key < nd_[p].key;
    }

    void grow() {
        const int32_t old_n = (int32_t)bins_.size();
        const int32_t n = old_n ? old_n * 2 : 16;
        threshold_ = n / 4 * 3;
        std::vector<int32_t> old(n, NIL);
        old.swap(bins_);
        for (int32_t j = 0; j < old_n; ++j) {
            const int32_t head = old[j];
            if (head == NIL) continue;
            if (nd_[head].next == NIL) { bins_[bin_of(nd_[head].hash)] = head; continue; }
            // split in order into j (bit clear) and j + old_n (bit set)
            int32_t h2[2] = {NIL, NIL}, t2[2] = {NIL, NIL}, c2[2] = {0, 0};
            const bool tree = nd_[head].tree;
            for (int32_t e = head, nx; e != NIL; e = nx) {
                nx = nd_[e].next;
                const int side = (nd_[e].hash & old_n) ? 1 : 0;
                nd_[e].next = NIL;
                if (tree) nd_[e].prev = t2[side];
                if (t2[side] == NIL) h2[side] = e; else nd_[t2[side]].next = e;
                t2[side] = e;
                ++c2[side];
            }
            for (int side = 0; side < 2; ++side) {
                if (h2[side] == NIL) continue;
                bins_[j + side * old_n] = h2[side];
                if (!tree) continue;
                if (c2[side] <= 6) to_list(h2[side]);
                else if (h2[1 - side] != NIL) build_tree(h2[side]);
            }
        }
    }

    void to_list(int32_t head) {
        for (int32_t e = head; e != NIL; e = nd_[e].next) {
            N& z = nd_[e];
            z.tree = z.red = false;
            z.prev = z.up = z.lo = z.hi = NIL;
        }
    }

    void make_tree_bin(int32_t h) {
        if (bins_.size() < 64) { grow(); return; }
        const int32_t head = bins_[bin_of(h)];
        int32_t last = NIL;
        for (int32_t e = head; e != NIL; e = nd_[e].next) {
            N& z = nd_[e];
            z.tree = true;
            z.red = false;
            z.up = z.lo = z.hi = NIL;
            z.prev = last;
            last = e;
        }
        build_tree(head);
    }

    // red-black tree over the bin's list, inserted in list order; the root then leads the list
    void build_tree(int32_t head) {
        int32_t root = NIL;
        for (int32_t x = head, nx; x != NIL; x = nx) {
            nx = nd_[x].next;
            nd_[x].lo = nd_[x].hi = NIL;
            if (root == NIL) { nd_[x].up = NIL; nd_[x].red = false; root = x; continue; }
            int32_t p = root;
            for (;;) {
                const bool left = goes_left(x, p);
                const int32_t c = left ? nd_[p].lo : nd_[p].hi;
                if (c != NIL) { p = c; continue; }
                nd_[x].up = p;
                (left ? nd_[p].lo : nd_[p].hi) = x;
                root = fix_insert(root, x);
                break;
            }
        }
        root_first(root);
    }

    int32_t root_from(int32_t e) const {
        while (nd_[e].up != NIL) e = nd_[e].up;
        return e;
    }

    void tree_insert(int32_t head, int32_t x) {
        const int32_t root = nd_[head].up != NIL ? root_from(head) : head;
        int32_t p = root;
        for (;;) {
            const bool left = goes_left(x, p);
            const int32_t c = left ? nd_[p].lo : nd_[p].hi;
            if (c != NIL) { p = c; continue; }
            const int32_t pn = nd_[p].next;
            N& z = nd_[x];
            z.tree = true;
            z.next = pn;
            (left ? nd_[p].lo : nd_[p].hi) = x;
            nd_[p].next = x;
            z.up = z.prev = p;
            if (pn != NIL) nd_[pn].prev = x;
            root_first(fix_insert(root, x));
            return;
        }
    }

    void root_first(int32_t root) {
        if (root == NIL) return;
        const int32_t b = bin_of(nd_[root].hash);
        const int32_t first = bins_[b];
        if (first == root) return;
        bins_[b] = root;
        const int32_t rp = nd_[root].prev, rn = nd_[root].next;
        if (rn != NIL) nd_[rn].prev = rp;
        if (rp != NIL) nd_[rp].next = rn;
        if (first != NIL) nd_[first].prev = root;
        nd_[root].next = first;
        nd_[root].prev = NIL;
    }

    bool red(int32_t e) const { return e != NIL && nd_[e].red; }

    int32_t rot_left(int32_t root, int32_t p) {
        if (p == NIL || nd_[p].hi == NIL) return root;
        const int32_t r = nd_[p].hi;
        const int32_t rl = nd_[p].hi = nd_[r].lo;
        if (rl != NIL) nd_[rl].up = p;
        const int32_t pp = nd_[r].up = nd_[p].up;
        if (pp == NIL) { root = r; nd_[r].red = false; }
        else if (nd_[pp].lo == p) nd_[pp].lo = r;
        else nd_[pp].hi = r;
        nd_[r].lo = p;
        nd_[p].up = r;
        return root;
    }

    int32_t rot_right(int32_t root, int32_t p) {
        if (p == NIL || nd_[p].lo == NIL) return root;
        const int32_t l = nd_[p].lo;
        const int32_t lr = nd_[p].lo = nd_[l].hi;
        if (lr != NIL) nd_[lr].up = p;
        const int32_t pp = nd_[l].up = nd_[p].up;
        if (pp == NIL) { root = l; nd_[l].red = false; }
        else if (nd_[pp].hi == p) nd_[pp].hi = l;
        else nd_[pp].lo = l;
        nd_[l].hi = p;
        nd_[p].up = l;
        return root;
    }

    int32_t fix_insert(int32_t root, int32_t x) {
        nd_[x].red = true;
        for (;;) {
            int32_t xp = nd_[x].up;
            if (xp == NIL) { nd_[x].red = false; return x; }
            int32_t xpp;
            if (!nd_[xp].red || (xpp = nd_[xp].up) == NIL) return root;
            const int32_t xppl = nd_[xpp].lo;
            if (xp == xppl) {
                const int32_t u = nd_[xpp].hi;
                if (red(u)) {
                    nd_[u].red = nd_[xp].red = false;
                    nd_[xpp].red = true;
                    x = xpp;
                    continue;
                }
                if (x == nd_[xp].hi) {
                    x = xp;
                    root = rot_left(root, x);
                    xp = nd_[x].up;
                    xpp = xp == NIL ? NIL : nd_[xp].up;
                }
                if (xp != NIL) {
                    nd_[xp].red = false;
                    if (xpp != NIL) { nd_[xpp].red = true; root = rot_right(root, xpp); }
                }
            } else {
                if (red(xppl)) {
                    nd_[xppl].red = nd_[xp].red = false;
                    nd_[xpp].red = true;
                    x = xpp;
                    continue;
                }
                if (x == nd_[xp].lo) {
                    x = xp;
                    root = rot_right(root, x);
                    xp = nd_[x].up;
                    xpp = xp == NIL ? NIL : nd_[xp].up;
                }
                if (xp != NIL) {
                    nd_[xp].red = false;
                    if (xpp != NIL) { nd_[xpp].red = true; root = rot_left(root, xpp); }
                }
            }
        }
    }

    int32_t fix_erase(int32_t root, int32_t x) {
        for (;;) {
            if (x == NIL || x == root) return root;
            int32_t xp = nd_[x].up;
            if (xp == NIL) { nd_[x].red = false; return x; }
            if (nd_[x].red) { nd_[x].red = false; return root; }
            if (nd_[xp].lo == x) {
                int32_t s = nd_[xp].hi;
                if (red(s)) {
                    nd_[s].red = false;
                    nd_[xp].red = true;
                    root = rot_left(root, xp);
                    xp = nd_[x].up;
                    s = xp == NIL ? NIL : nd_[xp].hi;
                }
                if (s == NIL) { x = xp; continue; }
                if (!red(nd_[s].hi) && !red(nd_[s].lo)) { nd_[s].red = true; x = xp; continue; }
                if (!red(nd_[s].hi)) {
                    if (nd_[s].lo != NIL) nd_[nd_[s].lo].red = false;
                    nd_[s].red = true;
                    root = rot_right(root, s);
                    xp = nd_[x].up;
                    s = xp == NIL ? NIL : nd_[xp].hi;
                }
                if (s != NIL) {
                    nd_[s].red = xp == NIL ? false : nd_[xp].red;
                    if (nd_[s].hi != NIL) nd_[nd_[s].hi].red = false;
                }
                if (xp != NIL) { nd_[xp].red = false; root = rot_left(root, xp); }
                x = root;
            } else {
                int32_t s = nd_[xp].lo;
                if (red(s)) {
                    nd_[s].red = false;
                    nd_[xp].red = true;
                    root = rot_right(root, xp);
                    xp = nd_[x].up;
                    s = xp == NIL ? NIL : nd_[xp].lo;
                }
                if (s == NIL) { x = xp; continue; }
                if (!red(nd_[s].lo) && !red(nd_[s].hi)) { nd_[s].red = true; x = xp; continue; }
                if (!red(nd_[s].lo)) {
                    if (nd_[s].hi != NIL) nd_[nd_[s].hi].red = false;
                    nd_[s].red = true;
                    root = rot_left(root, s);
                    xp = nd_[x].up;
                    s = xp == NIL ? NIL : nd_[xp].lo;
                }
                if (s != NIL) {
                    nd_[s].red = xp == NIL ? false : nd_[xp].red;
                    if (nd_[s].lo != NIL) nd_[nd_[s].lo].red = false;
                }
                if (xp != NIL) { nd_[xp].red = false; root = rot_right(root, xp); }
                x = root;
            }
        }
    }

    void tree_erase(int32_t p) {
        const int32_t b = bin_of(nd_[p].hash);
        int32_t first = bins_[b];
        int32_t root = first;
        const int32_t succ = nd_[p].next, pred = nd_[p].prev;
        if (pred == NIL) bins_[b] = first = succ;
        else nd_[pred].next = succ;
        if (succ != NIL) nd_[succ].prev = pred;
        if (first == NIL) return;
        if (nd_[root].up != NIL) root = root_from(root);
        if (nd_[root].hi == NIL || nd_[root].lo == NIL || nd_[nd_[root].lo].lo == NIL) {
            to_list(first);
            return;
        }
        const int32_t pl = nd_[p].lo, pr = nd_[p].hi;
        int32_t rep;
        if (pl != NIL && pr != NIL) {
            int32_t s = pr;
            while (nd_[s].lo != NIL) s = nd_[s].lo;
            std::swap(nd_[s].red, nd_[p].red);
            const int32_t sr = nd_[s].hi, pp = nd_[p].up;
            if (s == pr) {
                nd_[p].up = s;
                nd_[s].hi = p;
            } else {
                const int32_t sp = nd_[s].up;
                nd_[p].up = sp;
                if (sp != NIL) (s == nd_[sp].lo ? nd_[sp].lo : nd_[sp].hi) = p;
                nd_[s].hi = pr;
                nd_[pr].up = s;
            }
            nd_[p].lo = NIL;
            nd_[p].hi = sr;
            if (sr != NIL) nd_[sr].up = p;
            nd_[s].lo = pl;
            nd_[pl].up = s;
            nd_[s].up = pp;
            if (pp == NIL) root = s;
            else if (p == nd_[pp].lo) nd_[pp].lo = s;
            else nd_[pp].hi = s;
            rep = sr != NIL ? sr : p;
        } else {
            rep = pl != NIL ? pl : (pr != NIL ? pr : p);
        }
        if (rep != p) {
            const int32_t pp = nd_[rep].up = nd_[p].up;
            if (pp == NIL) { root = rep; nd_[rep].red = false; }
            else if (p == nd_[pp].lo) nd_[pp].lo = rep;
            else nd_[pp].hi = rep;
            nd_[p].lo = nd_[p].hi = nd_[p].up = NIL;
        }
        if (!nd_[p].red) fix_erase(root, rep);
        if (rep == p) {
            const int32_t pp = nd_[p].up;
            nd_[p].up = NIL;
            if (pp != NIL) {
                if (p == nd_[pp].lo) nd_[pp].lo = NIL;
                else if (p == nd_[pp].hi) nd_[pp].hi = NIL;
            }
        }
    }
};

}  // namespace shj
