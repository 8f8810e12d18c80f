/* oracle.h — C API of the CPU restatement (TEST INFRASTRUCTURE ONLY; see siddhi_oracle.cpp).
 * Same descriptor / batch / output structs as include/siddhi_hip.h so the parity tests drive both
 * libraries with identical inputs. */
#ifndef SIDDHI_ORACLE_H
#define SIDDHI_ORACLE_H
#include "../include/siddhi_hip.h"
#ifdef __cplusplus
extern "C" {
#endif
const char* or_last_error(void);
void* or_query_create(const sh_query_desc* desc);
void or_query_destroy(void* q);
int or_query_set_output_rate(void* q, int32_t kind, int64_t n);
int or_query_set_ext_timeout(void* q, int64_t ms);
int or_query_set_ext_replace_ts(void* q, int32_t on);
int or_query_rep_ts_attr(void* q, const int64_t** values, int64_t* n);
int or_query_set_strings(void* q, int32_t col, int64_t first_id, int64_t n, const uint16_t* units,
                         const int64_t* offsets);
int or_push(void* q, const sh_batch* b, const sh_out** out);
int or_advance_time(void* q, int64_t now, const sh_out** out);
void* or_aggregation_create(const sh_aggregation_desc* desc);
void or_aggregation_destroy(void* a);
int or_aggregation_push(void* a, const sh_batch* b);
int or_aggregation_advance_time(void* a, int64_t now);
int or_aggregation_table(void* a, int32_t duration, const sh_out** out);
int or_aggregation_find(void* a, int32_t per, int64_t start, int64_t end, const sh_out** out);
#ifdef __cplusplus
}
#endif
#endif
