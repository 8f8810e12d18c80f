// sh_wide.h — group keys wider than one window key (GroupByKeyGenerator.java:63-73 joins any number of
// group-by attributes into one key; QuerySelector groups by it).
//
// A window keys its state by one u64: one column of any type, or two 32-bit columns. Every other
// combination — three or more columns, or a long / double beside another column — is interned on the
// device into one 32-bit id per distinct key, and the window is keyed by that id (a synthetic dictionary
// column past the stream's own). The id is built by a chain of two-component interning levels:
//   a 64-bit column first gets its own level (value -> id), so every component is 32 bits;
//   level 0 interns (c0, c1), level j interns (id of level j-1, c_j+1) ... the last level's slot is the id.
// Events the filter drops get no id (kNoId through the chain, 0 in the window's column: the window
// never reads a dropped event's key). Output rows map ids back to the group-by values by walking the
// chain backwards (k_wide_decode), in the encoding sh_out reports keys.
#pragma once
#include <vector>

#include "sh_runtime.h"

namespace shd {

constexpr int kWideLevels = 2 * SH_MAX_GROUP;
constexpr u32 kNoId = 0xFFFFFFFFu;

// one interning level on the device: its table and key plan over a 2-column view (cs2) whose columns are
// a stream column or an earlier level's ids; where each component goes when decoding
struct WideLevel {
    KeyTable t;
    KeyPlan kp;          // over the level's own 2-column ColSet (col 0, col 1)
    int src[kKeyParts];  // >= 0: stream column; < 0: ids of level (-src - 1)
    int out[kKeyParts];  // >= 0: group-by output position; < 0: an earlier level's id (-out - 1)
};
struct WideDev {
    int nl;
    int last;  // level whose slot is the final id
    WideLevel lv[kWideLevels];
};

void launch_wide_level(hipStream_t s, ColSet full, FilterProg f, int first, ColSet cs2, const WideLevel& lv,
                       const u32* prev, int last, i64 n, u32* ids);
void launch_wide_decode(hipStream_t s, const WideDev& w, const i64* ids, i64 n, i64* out);

}  // namespace shd

struct WideKeys {
    int n = 0;  // group-by columns
    int col[SH_MAX_GROUP] = {};
    int type[SH_MAX_GROUP] = {};
    int nl = 0;
    shd::WideLevel lv[shd::kWideLevels] = {};
    KeyTableHost tab[shd::kWideLevels];
    DevBuf ids[shd::kWideLevels];
    // needed when the window's own key plan cannot take these columns
    static bool needed(int n_group, const int32_t* group, const int32_t* types);
    // the chain for `n_group` columns; every level's table holds `capacity` distinct prefixes
    int init(int n_group, const int32_t* group, int n_cols, const int32_t* types, int64_t capacity);
    // the window's key capacity: the final ids lie in [0, id_space())
    int64_t id_space() const { return (int64_t)tab[nl - 1].size_ + 1; }
    // every event's id (filter-passing events; 0 for the others) into the returned device column
    int intern(hipStream_t s, const shd::ColSet& full, const shd::FilterProg& f, int64_t n, const uint32_t** out);
    // rows' ids -> [n_group][n] group-by values (device)
    int decode(hipStream_t s, const int64_t* ids, int64_t n, int64_t* out);
    shd::WideDev dev() const;
    // checkpoint: every level's keys; load refuses a blob of another shape
    int save(std::vector<uint8_t>& blob, hipStream_t s);
    int load(const uint8_t* p, size_t len, size_t& off, hipStream_t s);
};
