// jhashmap.h — java.util.HashMap<String, V> of JDK 8 (the reference's build target, pom.xml:809),
// restated for its ITERATION ORDER. TEST INFRASTRUCTURE ONLY (part of the oracle, see siddhi_oracle.cpp).
//
// Why: Scheduler.onTimeChange (core/util/Scheduler.java:71-104) walks
// PartitionStateHolder.states (a HashMap<String, Map<String, State>> keyed by the partition key's
// toString(), PartitionStateHolder.java:36,46) and puts every due SchedulerState into a TreeMultimap
// whose values all compare equal (Scheduler.java:363-366): of several partitions due at the same time
// only the FIRST IN HASHMAP ITERATION ORDER fires in that call. That order is a function of the keys'
// String.hashCode and of the map's history, restated here operation by operation:
//  * computeIfAbsent (HashMap.computeIfAbsent, JDK 8): resize first when size > threshold (also when the
//    key is present), a new key is linked at the HEAD of its bin, a bin that already held >= 7 nodes is
//    treeified (or the table resized while it is shorter than 64);
//  * iterator remove (HashMap.removeNode with movable = false, used by returnAllStates :133-161);
//  * resize: capacity 16, doubling when size exceeds 0.75 capacity, never shrinking; bins split into
//    lo / hi lists in order (TreeNode.split: untreeify at <= 6, re-treeify otherwise);
//  * tree bins: red-black trees ordered by (spread hash, String.compareTo) whose `next` links are the
//    iteration order: a node is linked after its tree parent, the root is moved to the bin's front
//    (putTreeVal, treeify, moveRootToFront, balanceInsertion / balanceDeletion, removeTreeNode).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace jhm {

// String.hashCode over the UTF-16 code units
inline int32_t string_hash(const std::u16string& s) {
    uint32_t h = 0;
    for (char16_t c : s) h = 31u * h + (uint32_t)c;
    return (int32_t)h;
}
// HashMap.hash: h ^ (h >>> 16)
inline int32_t spread(int32_t h) { return h ^ (int32_t)((uint32_t)h >> 16); }

template <class V>
class HashMap {
   public:
    struct Node {
        int32_t hash;
        std::u16string key;
        V value;
        Node* next = nullptr;
        bool tree = false;  // TreeNode
        Node *parent = nullptr, *left = nullptr, *right = nullptr, *prev = nullptr;
        bool red = false;
    };

    ~HashMap() {
        for (auto& kv : nodes_) delete kv.second;
    }
    int size() const { return size_; }
    int capacity() const { return (int)tab_.size(); }
    bool contains(const std::u16string& k) const { return nodes_.count(k) != 0; }

    // HashMap.computeIfAbsent(key, k -> value) (JDK 8)
    void compute_if_absent(const std::u16string& key, const V& value) {
        const int32_t h = spread(string_hash(key));
        if (size_ > threshold_ || tab_.empty()) resize();
        const int n = (int)tab_.size(), i = (n - 1) & h;
        Node* first = tab_[i];
        int bin_count = 0;
        Node* t = nullptr;
        if (first) {
            if (first->tree) {
                t = first;
                if (nodes_.count(key)) return;  // getTreeNode found it
            } else {
                for (Node* e = first; e; e = e->next) {
                    if (e->hash == h && e->key == key) return;
                    ++bin_count;
                }
            }
        }
        Node* x = new Node();
        x->hash = h;
        x->key = key;
        x->value = value;
        nodes_[key] = x;
        if (t) {
            put_tree_val(t, x);
        } else {
            x->next = first;
            tab_[i] = x;
            if (bin_count >= 7) treeify_bin(h);
        }
        ++size_;
    }

    // HashMap.removeNode(hash, key, null, false, movable = false): HashIterator.remove
    void remove(const std::u16string& key) {
        auto it = nodes_.find(key);
        if (it == nodes_.end()) return;
        Node* node = it->second;
        const int i = ((int)tab_.size() - 1) & node->hash;
        if (node->tree) {
            remove_tree_node(node);
        } else if (tab_[i] == node) {
            tab_[i] = node->next;
        } else {
            Node* p = tab_[i];
            while (p->next != node) p = p->next;
            p->next = node->next;
        }
        nodes_.erase(it);
        delete node;
        --size_;
    }

    int tree_bins() const {  // diagnostics for tests
        int n = 0;
        for (Node* b : tab_) n += b && b->tree;
        return n;
    }

    // entries in iteration order (HashIterator: bins 0..n-1, each along `next`)
    template <class F>
    void for_each(F f) const {
        for (Node* b : tab_)
            for (Node* e = b; e; e = e->next) f(e->key, e->value);
    }

   private:
    std::vector<Node*> tab_;
    int size_ = 0, threshold_ = 0;
    std::unordered_map<std::u16string, Node*> nodes_;

    // HashMap.resize
    void resize() {
        const int old_cap = (int)tab_.size();
        const int new_cap = old_cap == 0 ? 16 : old_cap * 2;
        threshold_ = (int)(new_cap * 0.75f);
        std::vector<Node*> old;
        old.swap(tab_);
        tab_.assign((size_t)new_cap, nullptr);
        for (int j = 0; j < old_cap; ++j) {
            Node* e = old[j];
            if (!e) continue;
            if (!e->next) {
                tab_[e->hash & (new_cap - 1)] = e;
            } else if (e->tree) {
                split(e, j, old_cap);
            } else {
                Node *lo_h = nullptr, *lo_t = nullptr, *hi_h = nullptr, *hi_t = nullptr;
                for (Node* nx; e; e = nx) {
                    nx = e->next;
                    if ((e->hash & old_cap) == 0) {
                        if (!lo_t) lo_h = e; else lo_t->next = e;
                        lo_t = e;
                    } else {
                        if (!hi_t) hi_h = e; else hi_t->next = e;
                        hi_t = e;
                    }
                }
                if (lo_t) { lo_t->next = nullptr; tab_[j] = lo_h; }
                if (hi_t) { hi_t->next = nullptr; tab_[j + old_cap] = hi_h; }
            }
        }
    }

    // HashMap.treeifyBin
    void treeify_bin(int32_t hash) {
        if (tab_.size() < 64) { resize(); return; }
        const int index = ((int)tab_.size() - 1) & hash;
        Node* hd = tab_[index];
        if (!hd) return;
        Node* tl = nullptr;
        for (Node* e = hd; e; e = e->next) {  // replacementTreeNode, in order
            e->tree = true;
            e->parent = e->left = e->right = nullptr;
            e->red = false;
            e->prev = tl;
            tl = e;
        }
        treeify(hd);
    }

    static int dir_of(const Node* x, const Node* p) {  // hash, then String.compareTo (keys distinct)
        if (p->hash > x->hash) return -1;
        if (p->hash < x->hash) return 1;
        return x->key.compare(p->key) < 0 ? -1 : 1;
    }

    // TreeNode.treeify: the list from `head`, in order, into a red-black tree
    void treeify(Node* head) {
        Node* root = nullptr;
        for (Node *x = head, *nx; x; x = nx) {
            nx = x->next;
            x->left = x->right = nullptr;
            if (!root) {
                x->parent = nullptr;
                x->red = false;
                root = x;
                continue;
            }
            for (Node* p = root;;) {
                const int dir = dir_of(x, p);
                Node* xp = p;
                if (!(p = dir <= 0 ? p->left : p->right)) {
                    x->parent = xp;
                    if (dir <= 0) xp->left = x; else xp->right = x;
                    root = balance_insertion(root, x);
                    break;
                }
            }
        }
        move_root_to_front(root);
    }

    // TreeNode.untreeify: plain nodes in `next` order
    static void untreeify(Node* head) {
        for (Node* e = head; e; e = e->next) {
            e->tree = false;
            e->parent = e->left = e->right = e->prev = nullptr;
            e->red = false;
        }
    }

    static Node* root_of(Node* p) {
        while (p->parent) p = p->parent;
        return p;
    }

    // TreeNode.putTreeVal for a key known to be absent
    void put_tree_val(Node* bin_first, Node* x) {
        Node* root = bin_first->parent ? root_of(bin_first) : bin_first;
        for (Node* p = root;;) {
            const int dir = dir_of(x, p);
            Node* xp = p;
            if (!(p = dir <= 0 ? p->left : p->right)) {
                Node* xpn = xp->next;
                x->tree = true;
                x->next = xpn;
                if (dir <= 0) xp->left = x; else xp->right = x;
                xp->next = x;
                x->parent = x->prev = xp;
                if (xpn) xpn->prev = x;
                move_root_to_front(balance_insertion(root, x));
                return;
            }
        }
    }

    // TreeNode.moveRootToFront
    void move_root_to_front(Node* root) {
        if (!root || tab_.empty()) return;
        const int index = ((int)tab_.size() - 1) & root->hash;
        Node* first = tab_[index];
        if (root == first) return;
        tab_[index] = root;
        Node* rp = root->prev;
        Node* rn = root->next;
        if (rn) rn->prev = rp;
        if (rp) rp->next = rn;
        if (first) first->prev = root;
        root->next = first;
        root->prev = nullptr;
    }

    // TreeNode.split (resize of a tree bin)
    void split(Node* b, int index, int bit) {
        Node *lo_h = nullptr, *lo_t = nullptr, *hi_h = nullptr, *hi_t = nullptr;
        int lc = 0, hc = 0;
        for (Node *e = b, *nx; e; e = nx) {
            nx = e->next;
            e->next = nullptr;
            if ((e->hash & bit) == 0) {
                if (!(e->prev = lo_t)) lo_h = e; else lo_t->next = e;
                lo_t = e;
                ++lc;
            } else {
                if (!(e->prev = hi_t)) hi_h = e; else hi_t->next = e;
                hi_t = e;
                ++hc;
            }
        }
        if (lo_h) {
            if (lc <= 6) { untreeify(lo_h); tab_[index] = lo_h; }
            else { tab_[index] = lo_h; if (hi_h) treeify(lo_h); }
        }
        if (hi_h) {
            if (hc <= 6) { untreeify(hi_h); tab_[index + bit] = hi_h; }
            else { tab_[index + bit] = hi_h; if (lo_h) treeify(hi_h); }
        }
    }

    static Node* rotate_left(Node* root, Node* p) {
        Node *r, *pp, *rl;
        if (p && (r = p->right)) {
            if ((rl = p->right = r->left)) rl->parent = p;
            if (!(pp = r->parent = p->parent)) (root = r)->red = false;
            else if (pp->left == p) pp->left = r;
            else pp->right = r;
            r->left = p;
            p->parent = r;
        }
        return root;
    }
    static Node* rotate_right(Node* root, Node* p) {
        Node *l, *pp, *lr;
        if (p && (l = p->left)) {
            if ((lr = p->left = l->right)) lr->parent = p;
            if (!(pp = l->parent = p->parent)) (root = l)->red = false;
            else if (pp->right == p) pp->right = l;
            else pp->left = l;
            l->right = p;
            p->parent = l;
        }
        return root;
    }

    // TreeNode.balanceInsertion
    static Node* balance_insertion(Node* root, Node* x) {
        x->red = true;
        for (Node *xp, *xpp, *xppl, *xppr;;) {
            if (!(xp = x->parent)) { x->red = false; return x; }
            if (!xp->red || !(xpp = xp->parent)) return root;
            if (xp == (xppl = xpp->left)) {
                if ((xppr = xpp->right) && xppr->red) {
                    xppr->red = false; xp->red = false; xpp->red = true; x = xpp;
                } else {
                    if (x == xp->right) {
                        root = rotate_left(root, x = xp);
                        xpp = (xp = x->parent) ? xp->parent : nullptr;
                    }
                    if (xp) {
                        xp->red = false;
                        if (xpp) { xpp->red = true; root = rotate_right(root, xpp); }
                    }
                }
            } else {
                if (xppl && xppl->red) {
                    xppl->red = false; xp->red = false; xpp->red = true; x = xpp;
                } else {
                    if (x == xp->left) {
                        root = rotate_right(root, x = xp);
                        xpp = (xp = x->parent) ? xp->parent : nullptr;
                    }
                    if (xp) {
                        xp->red = false;
                        if (xpp) { xpp->red = true; root = rotate_left(root, xpp); }
                    }
                }
            }
        }
    }

    // TreeNode.balanceDeletion
    static Node* balance_deletion(Node* root, Node* x) {
        for (Node *xp, *xpl, *xpr;;) {
            if (!x || x == root) return root;
            if (!(xp = x->parent)) { x->red = false; return x; }
            if (x->red) { x->red = false; return root; }
            if ((xpl = xp->left) == x) {
                if ((xpr = xp->right) && xpr->red) {
                    xpr->red = false; xp->red = true;
                    root = rotate_left(root, xp);
                    xpr = (xp = x->parent) ? xp->right : nullptr;
                }
                if (!xpr) { x = xp; continue; }
                Node *sl = xpr->left, *sr = xpr->right;
                if ((!sr || !sr->red) && (!sl || !sl->red)) { xpr->red = true; x = xp; continue; }
                if (!sr || !sr->red) {
                    if (sl) sl->red = false;
                    xpr->red = true;
                    root = rotate_right(root, xpr);
                    xpr = (xp = x->parent) ? xp->right : nullptr;
                }
                if (xpr) {
                    xpr->red = xp ? xp->red : false;
                    if ((sr = xpr->right)) sr->red = false;
                }
                if (xp) { xp->red = false; root = rotate_left(root, xp); }
                x = root;
            } else {
                if (xpl && xpl->red) {
                    xpl->red = false; xp->red = true;
                    root = rotate_right(root, xp);
                    xpl = (xp = x->parent) ? xp->left : nullptr;
                }
                if (!xpl) { x = xp; continue; }
                Node *sl = xpl->left, *sr = xpl->right;
                if ((!sl || !sl->red) && (!sr || !sr->red)) { xpl->red = true; x = xp; continue; }
                if (!sl || !sl->red) {
                    if (sr) sr->red = false;
                    xpl->red = true;
                    root = rotate_left(root, xpl);
                    xpl = (xp = x->parent) ? xp->left : nullptr;
                }
                if (xpl) {
                    xpl->red = xp ? xp->red : false;
                    if ((sl = xpl->left)) sl->red = false;
                }
                if (xp) { xp->red = false; root = rotate_right(root, xp); }
                x = root;
            }
        }
    }

    // TreeNode.removeTreeNode(map, tab, movable = false) — JDK 8: a tree left with no right child,
    // no left child or no left grandchild of the root becomes a list again
    void remove_tree_node(Node* p) {
        const int index = ((int)tab_.size() - 1) & p->hash;
        Node* first = tab_[index];
        Node* root = first;
        Node* succ = p->next;
        Node* pred = p->prev;
        if (!pred) tab_[index] = first = succ;
        else pred->next = succ;
        if (succ) succ->prev = pred;
        if (!first) return;
        if (root->parent) root = root_of(root);
        Node* rl;
        if (!root || !root->right || !(rl = root->left) || !rl->left) {
            untreeify(first);  // too small
            tab_[index] = first;
            return;
        }
        Node *pl = p->left, *pr = p->right, *replacement;
        if (pl && pr) {
            Node *s = pr, *sl;
            while ((sl = s->left)) s = sl;
            const bool c = s->red;
            s->red = p->red;
            p->red = c;  // swap colours
            Node* sr = s->right;
            Node* pp = p->parent;
            if (s == pr) {  // p was s's direct parent
                p->parent = s;
                s->right = p;
            } else {
                Node* sp = s->parent;
                if ((p->parent = sp)) {
                    if (s == sp->left) sp->left = p; else sp->right = p;
                }
                if ((s->right = pr)) pr->parent = s;
            }
            p->left = nullptr;
            if ((p->right = sr)) sr->parent = p;
            if ((s->left = pl)) pl->parent = s;
            if (!(s->parent = pp)) root = s;
            else if (p == pp->left) pp->left = s;
            else pp->right = s;
            replacement = sr ? sr : p;
        } else if (pl) {
            replacement = pl;
        } else if (pr) {
            replacement = pr;
        } else {
            replacement = p;
        }
        if (replacement != p) {
            Node* pp = replacement->parent = p->parent;
            if (!pp) (root = replacement)->red = false;
            else if (p == pp->left) pp->left = replacement;
            else pp->right = replacement;
            p->left = p->right = p->parent = nullptr;
        }
        Node* r = p->red ? root : balance_deletion(root, replacement);
        (void)r;  // movable == false: the root is not moved to the front
        if (replacement == p) {  // detach
            Node* pp = p->parent;
            p->parent = nullptr;
            if (pp) {
                if (p == pp->left) pp->left = nullptr;
                else if (p == pp->right) pp->right = nullptr;
            }
        }
    }
};

// String.valueOf(x) of the partition key types the oracle restates (ValuePartitionExecutor :34-40)
inline std::u16string decimal(int64_t v) {
    std::string s = std::to_string(v);
    return std::u16string(s.begin(), s.end());
}

// String.valueOf(x) of a double / float key: Double.toString / Float.toString as the JDK 8 javadoc specifies
// them — the fewest significant digits (at least one after the point) that tell the value apart from its
// neighbours of the type, searched here by printing with 1, 2, ... 17 digits until the text reads back as
// the value (printf rounds to nearest, so the text found is also the nearest of its length); when one digit
// suffices a two-digit text that reads back and lies nearer wins (Double.MIN_VALUE prints "4.9E-324").
// Plain notation for 1e-3 <= |x| < 1e7, else "d.dddE<exponent>". (JDK 8's FloatingDecimal prints more digits
// for a few values, JDK-4511638; those are not restated.)
inline std::u16string fp_decimal(double x, bool is_float) {
    if (std::isnan(x)) return u"NaN";
    if (std::isinf(x)) return x < 0 ? u"-Infinity" : u"Infinity";
    if (x == 0.0) return std::signbit(x) ? u"-0.0" : u"0.0";
    auto reads_back = [&](const char* t) {
        return is_float ? (std::strtof(t, nullptr) == (float)x) : (std::strtod(t, nullptr) == x);
    };
    char t[64];
    int p = 0;
    for (; p < 17; p++) {
        std::snprintf(t, sizeof t, "%.*e", p, x);
        if (reads_back(t)) break;
    }
    if (p == 0) {
        char u[64];
        std::snprintf(u, sizeof u, "%.1e", x);
        // (distances in long double: both texts read back as x itself)
        const long double lx = x;
        if (reads_back(u) && std::fabs(std::strtold(u, nullptr) - lx) < std::fabs(std::strtold(t, nullptr) - lx))
            std::memcpy(t, u, sizeof t);
    }
    // mantissa digits (trailing zeros dropped) and the decimal exponent
    std::string m;
    const char* e = std::strchr(t, 'e');
    for (const char* c = t; c < e; c++)
        if (*c >= '0' && *c <= '9') m += *c;
    while (m.size() > 1 && m.back() == '0') m.pop_back();
    const int ex = std::atoi(e + 1);
    std::string r = x < 0 ? "-" : "";
    const double ax = std::fabs(x);
    if (ax >= 1e-3 && ax < 1e7) {
        if (ex < 0) {
            r += "0." + std::string((size_t)(-ex - 1), '0') + m;
        } else {
            std::string ip = m.substr(0, std::min(m.size(), (size_t)ex + 1));
            ip.resize((size_t)ex + 1, '0');
            const std::string fp = m.size() > (size_t)ex + 1 ? m.substr((size_t)ex + 1) : "0";
            r += ip + "." + fp;
        }
    } else {
        r += m.substr(0, 1) + "." + (m.size() > 1 ? m.substr(1) : "0") + "E" + std::to_string(ex);
    }
    return std::u16string(r.begin(), r.end());
}

}  // namespace jhm
