"""Transcribe the reference's own TestNG known-answer cases into tests/golden/kat_reference.json.

Each case records the query, the exact sends of the Java test (timestamps added: the wall-clock
tests are transcribed to playback timestamps that reproduce the timer firing the test relies on),
and ONLY the expectations the Java test asserts (counts, values). Nothing here is computed by
the oracle: this file pins the oracle, it is not produced by it.

ctest/ = /root/reference/modules/siddhi-core/src/test/java/io/siddhi/core/
Run: python tests/golden/make_kat.py
"""
import json
import os

CASES = []


def case(**kw):
    CASES.append(kw)


CSE_FLOAT_INT = "symbol string, price float, volume int"
B = 1_000_000  # base timestamp for transcribed wall-clock sends
LOGIN = "timestamp long, ip string"

# ---------------------------------------------------------------- lengthBatch (LengthBatchWindowTestCase)
_six = [["IBM", 700.0, 1], ["WSO2", 60.5, 2], ["IBM", 700.0, 3], ["WSO2", 60.5, 4], ["IBM", 700.0, 5],
        ["WSO2", 60.5, 6]]
case(name="lengthBatch2_passthrough", source="ctest/query/window/LengthBatchWindowTestCase.java:89-132",
     schema=CSE_FLOAT_INT, query=dict(window="lengthBatch", param=4, output="current"),
     sends=[[[B + i] + r] for i, r in enumerate(_six)],
     expect=dict(in_count=4, in_order_col="volume", in_order=[1, 2, 3, 4]))
case(name="lengthBatch3_all_events", source="ctest/query/window/LengthBatchWindowTestCase.java:134-190",
     schema=CSE_FLOAT_INT, query=dict(window="lengthBatch", param=2, output="all"),
     sends=[[[B + i] + r] for i, r in enumerate(_six)],
     expect=dict(in_count=6, remove_count=4, in_order_col="volume", in_order=[1, 2, 3, 4, 5, 6],
                 remove_order=[1, 2, 3, 4]))
_lb4 = [["IBM", 10.0, 0], ["WSO2", 20.0, 1], ["IBM", 30.0, 0], ["WSO2", 40.0, 1], ["IBM", 50.0, 0],
        ["WSO2", 60.0, 1]]
# `select symbol, sum(price) as sumPrice, volume`: the Java test asserts sumPrice; symbol and volume
# are the batch's last event's (QuerySelector.processInBatchNoGroupBy keeps the chunk's last event),
# hand-traced here as rep_cols: WSO2 / 1 (the 4th event)
case(name="lengthBatch4_sum", source="ctest/query/window/LengthBatchWindowTestCase.java:192-234",
     schema=CSE_FLOAT_INT, query=dict(window="lengthBatch", param=4, aggs=[["sum", "price"]], output="current"),
     sends=[[[B + i] + r] for i, r in enumerate(_lb4)],
     expect=dict(in_count=1, remove_count=0, values=[[100.0]], rep_cols=[["volume", [1]], ["symbol", ["WSO2"]]]))
case(name="lengthBatch5_expired", source="ctest/query/window/LengthBatchWindowTestCase.java:236-277",
     schema=CSE_FLOAT_INT, query=dict(window="lengthBatch", param=2, output="expired"),
     sends=[[[B + i] + r] for i, r in enumerate(_six)],
     expect=dict(remove_count=4, in_count=0, remove_order=[1, 2, 3, 4]))
_lb6 = _lb4 + [["WSO2", 60.0, 1], ["IBM", 70.0, 0], ["WSO2", 80.0, 1]]
case(name="lengthBatch6_sum_all_events", source="ctest/query/window/LengthBatchWindowTestCase.java:279-327",
     schema=CSE_FLOAT_INT, query=dict(window="lengthBatch", param=4, aggs=[["sum", "price"]], output="all"),
     sends=[[[B + i] + r] for i, r in enumerate(_lb6)],
     expect=dict(in_count=2, values=[[100.0], [240.0]]))
_nine = _six + [["WSO2", 60.5, 4], ["IBM", 700.0, 5], ["WSO2", 60.5, 6]]
case(name="lengthBatch11_stream_current_count", source="ctest/query/window/LengthBatchWindowTestCase.java:534-590",
     schema=CSE_FLOAT_INT,
     query=dict(window="lengthBatch", param=4, stream_current=True, aggs=[["count", None]], output="current"),
     sends=[[[B + i] + r] for i, r in enumerate(_nine)],
     expect=dict(in_count=9, flush_sizes=[1] * 9, value_range=[0, 1, 4]))
case(name="lengthBatch12_stream_current_expired", source="ctest/query/window/LengthBatchWindowTestCase.java:592-646",
     schema=CSE_FLOAT_INT,
     query=dict(window="lengthBatch", param=4, stream_current=True, aggs=[["count", None]], output="expired"),
     sends=[[[B + i] + r] for i, r in enumerate(_nine)],
     expect=dict(total_count=2, flush_sizes=[1, 1], values=[[0], [0]]))

# ---------------------------------------------------------------- playback (PlaybackTestCase)
case(name="playback1_timeBatch", source="ctest/managment/PlaybackTestCase.java:48-107",
     schema=CSE_FLOAT_INT, query=dict(window="timeBatch", param=1000, output="all"),
     sends=[[[B, "IBM", 700.0, 0]], [[B + 500, "WSO2", 60.5, 1]], [[B + 1000, "GOOGLE", 85.0, 1]],
            [[B + 2000, "ORACLE", 90.5, 1]]],
     expect=dict(in_count=3, remove_count=2))
case(name="playback2_timeBatch_start", source="ctest/managment/PlaybackTestCase.java:109-169",
     schema=CSE_FLOAT_INT,
     query=dict(window="timeBatch", param=2000, start_time=0, aggs=[["sum", "price"]], output="current"),
     sends=[[[0, "IBM", 700.0, 0]], [[0, "WSO2", 60.5, 1]], [[8500, "WSO2", 60.5, 1]], [[8500, "II", 60.5, 1]],
            [[21500, "TT", 60.5, 1]], [[21500, "YY", 60.5, 1]], [[26500, "ZZ", 0.0, 0]]],
     expect=dict(in_count=3, remove_count=0))
case(name="playback7_time", source="ctest/managment/PlaybackTestCase.java:383-432",
     schema=CSE_FLOAT_INT, query=dict(window="time", param=2000, output="all"),
     sends=[[[B, "IBM", 700.0, 0]], [[B, "WSO2", 60.5, 1]], [[B + 2000, "GOOGLE", 0.0, 1]]],
     expect=dict(in_count=3, remove_count=2))

# ---------------------------------------------------------------- sliding max (MaxAggregatorExtensionTestCase)
# wall-clock sends at t and t+100, then the two expiry timers fire at t+1000 and t+1100
case(name="max_sliding_time", source="ctest/query/aggregator/MaxAggregatorExtensionTestCase.java:47-101",
     schema="price1 double, price2 double, price3 double",
     query=dict(window="time", param=1000, aggs=[["max", "price1"]], output="all"),
     sends=[[[B, 36.0, 36.75, 35.75]], [[B + 100, 37.88, 38.12, 37.62]], {"advance": B + 1000},
            {"advance": B + 1100}],
     expect=dict(total_count=4, values=[[36.0], [37.88], [37.88], [None]]))

# ---------------------------------------------------------------- externalTimeBatch (ExternalTimeBatchWindowTestCase)
# The window keys on an attribute; the (wall-clock) event timestamps of these tests never matter, so
# each send carries a distinct timestamp B + value that lets the checks map a row back to `value`.
E = "ctest/query/window/ExternalTimeBatchWindowTestCase.java"
_e1 = [10000, 11000, 12000, 13000, 14000, 15000, 16500, 17000, 18000, 19000, 20000, 20500, 22000, 25000]
case(name="externalTimeBatch_test1", source=E + ":225-285", schema="currentTime long, value int",
     query=dict(window="externalTimeBatch", param=5000, ts_attr="currentTime", output="current"),
     sends=[[[B + i + 1, t, i + 1]] for i, t in enumerate(_e1)],
     expect=dict(flush_count=3, flush_first_col=["value", [1, 6, 11]]))
case(name="externalTimeBatch_test2_start", source=E + ":287-323", schema="currentTime long, value int",
     query=dict(window="externalTimeBatch", param=5000, ts_attr="currentTime", start_time=1200, output="current"),
     sends=[[[B + i // 100, i + 10000, i // 100]] for i in range(0, 10000, 100)],
     expect=dict(flush_first_col=["value", [0, 12]], flush_last_col=["value", [11]]))
case(name="externalTimeBatch_test05_edge", source=E + ":99-141", schema="cpu int, timestamp long",
     query=dict(window="externalTimeBatch", param=10000, ts_attr="timestamp", aggs=[["avg", "cpu"], ["count", None]],
                output="current"),
     sends=[[[B + i, c, t]] for i, (c, t) in enumerate([(15, 0), (15, 10), (15, 20), (85, 10000), (85, 10010),
                                                        (85, 10020), (10000, 100000)])],
     expect=dict(in_count=2, flush_sizes=[1, 1], values=[[15.0, 3], [85.0, 3]]))

# externalTimeBatch(ts, T, start, timeout): the wall-clock tests send at w ms (Thread.sleep between
# sends), so each send's event timestamp is B + w and the scheduler's timeout timers fire as the
# clock passes them (ExternalTimeBatchWindowProcessor.process :256-275); a final advance stands for
# the last sleep
_sched = [10000, 11000, 12000, 13000, 14000, 15000, 16500, 17000, 18000, 19000, 20100, 20500, 22000, 25000,
          32000, 33000]
case(name="externalTimeBatch_scheduler_last_batch", source=E + ":325-392", schema="currentTime long, value int",
     query=dict(window="externalTimeBatch", param=5000, ts_attr="currentTime", start_time=0, timeout=6000,
                output="current"),
     sends=[[[B + 100 * i, t, i + 1]] for i, t in enumerate(_sched)] + [{"advance": B + 1500 + 6000}],
     expect=dict(flush_count=5, flush_first_col=["value", [1, 6, 11, 14, 15]]))


def _login(*ws):
    """(wall ms, timestamp attribute, ip suffix) sends of the LoginEvents tests."""
    return [[[B + w, t, "192.10.1." + str(x)]] for w, t, x in ws]


_L0 = 1366335800000
_t4 = [(0, 4341, 3), (0, 4342, 4), (0, 14341, 5), (0, 14345, 6), (0, 24341, 7)]
case(name="externalTimeBatch_w1_timeout", source=E + ":394-440", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=6000,
                aggs=[["count", None]], output="all"),
     sends=_login(*[(w, _L0 + t, x) for w, t, x in _t4]) + [{"advance": B + 1000}],
     expect=dict(in_count=2, remove_count=0))
case(name="externalTimeBatch_w2", source=E + ":442-490", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, x) for t, x in [(4341, 3), (4342, 4), (5340, 4), (14341, 5), (14345, 6),
                                                 (24341, 7)]]),
     expect=dict(in_count=2, remove_count=0))
case(name="externalTimeBatch_w3", source=E + ":492-540", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, x) for t, x in [(4341, 3), (4342, 4), (5341, 4), (14341, 5), (14345, 6),
                                                 (24341, 7)]]),
     expect=dict(in_count=3, remove_count=0))
case(name="externalTimeBatch_w4_timeout", source=E + ":542-591", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=6000,
                aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, x) for t, x in [(4341, 3), (4999, 4), (5000, 4), (5999, 5), (6000, 6),
                                                 (6001, 6), (24341, 7)]]) + [{"advance": B + 1000}],
     expect=dict(in_count=3, remove_count=0))
_w5 = [(4341, 3), (4599, 4), (4600, 5), (4607, 6)]
_w6 = _w5 + [(5599, 4), (5600, 5), (5607, 6)]
case(name="externalTimeBatch_w5_timeout", source=E + ":593-640", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=3000,
                aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, x) for t, x in _w5]) + [{"advance": B + 5000}],
     expect=dict(in_count=1, remove_count=0))
case(name="externalTimeBatch_w6_timeout", source=E + ":642-691", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=3000,
                aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, x) for t, x in _w6]) + [{"advance": B + 5000}],
     expect=dict(in_count=2, remove_count=0))
case(name="externalTimeBatch_w7_timeout_resend", source=E + ":693-747", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=2000,
                aggs=[["count", None]], output="all"),
     sends=_login(*([(0, _L0 + t, x) for t, x in _w6] + [(3000, _L0 + 5606, 7), (3000, _L0 + 5605, 8),
                                                          (6000, _L0 + 6606, 9), (6000, _L0 + 6690, 10)]))
     + [{"advance": B + 9000}],
     expect=dict(in_count=4, remove_count=0))
_w8 = ([(0, _L0 + t, x) for t, x in _w6] + [(2100, _L0 + 5606, 7), (2100, _L0 + 5605, 8), (4200, _L0 + 5606, 91),
                                           (4200, _L0 + 5605, 92), (4200, _L0 + 6606, 9), (4200, _L0 + 6690, 10)])
case(name="externalTimeBatch_w8_timeout_counts", source=E + ":749-815", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=2000,
                aggs=[["count", None]], output="all"),
     sends=_login(*_w8) + [{"advance": B + 7200}],
     expect=dict(in_count=5, remove_count=0, values=[[4], [3], [5], [7], [2]]))
case(name="externalTimeBatch_w10_timeout_current", source=E + ":884-950", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=2000,
                aggs=[["count", None]], output="current"),
     sends=_login(*_w8) + [{"advance": B + 7200}],
     expect=dict(in_count=5, remove_count=0, values=[[4], [3], [5], [7], [2]]))

# test17: externalTimeBatch(timestamp, 1 sec, 0, 100, false) — the 100 ms timeout sends the last
# batch during the final sleep; `select timestamp` shows each row's last event (not replaced: % 100 != 0)
_t17x = [4341, 4342, 5341, 14341, 14345, 24341, 24351, 24441]
case(name="externalTimeBatch_w17_timeout_not_replaced", source=E + ":1272-1330", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=100,
                aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, 3 + i) for i, t in enumerate(_t17x)]) + [{"advance": B + 1000}],
     expect=dict(in_count=4, remove_count=0, values=[[2], [1], [2], [3]],
                 rep_cols=[["timestamp", [_L0 + 4342, _L0 + 5341, _L0 + 14345, _L0 + 24441]]]))
# test15: externalTimeBatch(timestamp, 1 sec, timestamp, 100) — the start time from the first event's
# `timestamp` attribute (initTiming :319-322: endTime = start + 1 sec), no group-by, all events; the sends
# arrive within a millisecond and the 100 ms timeout fires in the final 1 s sleep (the last batch)
case(name="externalTimeBatch_w15_start_attr_timeout", source=E + ":1162-1211", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_attr="timestamp", timeout=100,
                aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, 3 + i) for i, t in enumerate(_t17x)]) + [{"advance": B + 1000}],
     expect=dict(in_count=4, remove_count=0, values=[[2], [1], [2], [3]],
                 rep_cols=[["timestamp", [_L0 + 4342, _L0 + 5341, _L0 + 14345, _L0 + 24441]]]))
# test16: the same with replaceTimestampWithBatchEndTime = true (5th parameter, :210-220): cloneAppend
# (:446-456) writes the batch's endTime into every kept event's timestamp attribute, so each row's
# `timestamp` is its batch end (% 100 == 0): 805000, 806000 (the crossing event gets the new endTime),
# 815000 and, at the timeout, 825000
case(name="externalTimeBatch_w16_timeout_replaced", source=E + ":1214-1270", schema=LOGIN,
     query=dict(window="externalTimeBatch", param=1000, ts_attr="timestamp", start_time=0, timeout=100,
                replace_ts=True, aggs=[["count", None]], output="all"),
     sends=_login(*[(0, _L0 + t, 3 + i) for i, t in enumerate(_t17x)]) + [{"advance": B + 1000}],
     expect=dict(in_count=4, remove_count=0, values=[[2], [1], [2], [3]],
                 rep_cols=[["timestamp", [_L0 + 5000, _L0 + 6000, _L0 + 15000, _L0 + 25000]]]))

# ---------------------------------------------------------------- externalTime (ExternalTimeWindowTestCase)
# sliding over the `timestamp` attribute: 804341/804342 expire at 814341, 814341/814345 at 824341
X = "ctest/query/window/ExternalTimeWindowTestCase.java"
case(name="externalTime_test1", source=X + ":49-95", schema="timestamp long, ip string",
     query=dict(window="externalTime", param=5000, ts_attr="timestamp", output="all"),
     sends=[[[B + i, t, ip]] for i, (t, ip) in enumerate([(1366335804341, "192.10.1.3"), (1366335804342, "192.10.1.4"),
                                                          (1366335814341, "192.10.1.5"), (1366335814345, "192.10.1.6"),
                                                          (1366335824341, "192.10.1.7")])],
     expect=dict(in_count=5, remove_count=4))

# ---------------------------------------------------------------- partitioned timeBatch (WindowPartitionTestCase)
case(name="partition5_timeBatch", source="ctest/query/partition/WindowPartitionTestCase.java:291-348",
     schema="symbol string, price double, volume int",
     query=dict(window="timeBatch", param=5000, partition="symbol", aggs=[["sum", "price"]], output="current"),
     sends=[[[B + i] + r] for i, r in enumerate([["IBM", 70.0, 100], ["WSO2", 700.0, 100], ["IBM", 100.0, 100],
                                                ["IBM", 200.0, 100], ["ORACLE", 75.6, 100],
                                                ["WSO2", 1000.0, 100], ["WSO2", 500.0, 100]])]
     + [{"advance": B + 7000}],
     expect=dict(in_count_max=7, remove_count=0, min_in_count=1, partition_values={"IBM": 370.0, "WSO2": 2200.0,
                                                                                    "ORACLE": 75.6}))

# partitioned lengthBatch(2) without group-by, `insert all events`: IBM's first batch (70, 100) and
# WSO2's (700, 1000) complete; IBM 200 stays open. Two events, 170.0 then 1700.0 (sum of the floats).
case(name="partition2_lengthBatch_all", source="ctest/query/partition/WindowPartitionTestCase.java:96-139",
     schema="symbol string, price float, volume int",
     query=dict(window="lengthBatch", param=2, partition="symbol", aggs=[["sum", "price"]], output="all"),
     sends=[[[B + i] + r] for i, r in enumerate([["IBM", 70.0, 100], ["WSO2", 700.0, 100], ["IBM", 100.0, 100],
                                                ["IBM", 200.0, 100], ["WSO2", 1000.0, 100]])],
     expect=dict(total_count=2, values=[[170.0], [1700.0]], rep_cols=[["symbol", ["IBM", "WSO2"]]]))

# partitioned time(1 sec) without group-by, `insert all events`, `default(sum(price), 0.0)`: the Java test
# sleeps between sends and lets the wall-clock scheduler expire each partition's events 1 s after they
# arrived; in playback those scheduler calls are TIMER calls at B+1000 (IBM 70), B+1100 (WSO2 700),
# B+1200 (IBM 100), B+4200 and B+4300. WSO2 rows: 700, 0.0, 1000, 0.0; IBM rows: 70, 170, 100, 0.0,
# 200, 0.0 (the callback counts them by symbol); default() turns the null sums into 0.0 (None here).
case(name="partition3_time_all", source="ctest/query/partition/WindowPartitionTestCase.java:141-216",
     schema="symbol string, price float, volume int",
     query=dict(window="time", param=1000, partition="symbol", aggs=[["sum", "price"]], output="all"),
     sends=[[[B, "IBM", 70.0, 100]], [[B + 100, "WSO2", 700.0, 100]], [[B + 200, "IBM", 100.0, 200]],
            {"advance": B + 1000}, {"advance": B + 1100}, {"advance": B + 1200},
            [[B + 3200, "IBM", 200.0, 300]], [[B + 3300, "WSO2", 1000.0, 100]],
            {"advance": B + 4200}, {"advance": B + 4300}],
     expect=dict(total_count=10, values=[[70.0], [700.0], [170.0], [100.0], [None], [None], [200.0], [1000.0],
                                         [None], [None]],
                 rep_cols=[["symbol", ["IBM", "WSO2", "IBM", "IBM", "WSO2", "IBM", "IBM", "WSO2", "IBM", "WSO2"]]]))

# partitioned lengthBatch(2, true) (stream.current.event), no group-by, `insert all events`: every event
# emits its partition's running sum; the third WSO2 and the third IBM event start a new batch (the chunk
# [expired batch, RESET, event] keeps only its last event, processInBatchNoGroupBy).
case(name="partition_lengthBatch_stream_current_all", source="ctest/query/partition/PartitionTestCase2.java:681-736",
     schema="ts long, symbol string, price int",
     query=dict(window="lengthBatch", param=2, partition="symbol", stream_current=True, aggs=[["sum", "price"]],
                output="all"),
     sends=[[[B + i] + r] for i, r in enumerate([[100, "IBM", 700], [101, "WSO2", 60], [101, "WSO2", 60],
                                                [1134, "WSO2", 60], [100, "IBM", 700], [1145, "IBM", 700]])],
     expect=dict(total_count=6, values=[[700], [60], [120], [60], [1400], [700]],
                 rep_cols=[["symbol", ["IBM", "WSO2", "WSO2", "WSO2", "IBM", "IBM"]]]))

# Scheduler tie rule, hand-traced (no reference test pins it; ctest/query/partition/WindowPartitionTestCase.java:
# 141-216 is the query shape). Five partitions are due at the same time B+1000; Scheduler.onTimeChange
# (core/util/Scheduler.java:71-104) walks PartitionStateHolder.states (HashMap<String, …>,
# PartitionStateHolder.java:36,46) and its TreeMultimap keeps ONE state per due time (values compare
# equal, :363-366), so each later send's call fires the next one, in HashMap iteration order:
#   String.hashCode   "WSO2" = 2674079 = 0x28CD9F   spread ^ (h >>> 16) = 0x28CDB7 -> bin 7 of 16
#                     "IBM"  = 72276   = 0x11A54    spread 0x11A55    -> bin 5
#                     "ORACLE" = 0x8B70F17E         spread 0x8B707A0E -> bin 14
#                     "Aa" = 65*31+97 = 2112 = "BB" = 66*31+66 (0x840, spread 0x840) -> bin 0
#   computeIfAbsent links a new key at the HEAD of its bin (JDK 8), so bin 0 reads BB, Aa.
#   Iteration: BB, Aa, IBM, WSO2, ORACLE (creation order was WSO2, IBM, ORACLE, Aa, BB).
# Each expiry empties its partition (sum null); the x partitions register B+2000.. and are never due.
_tie = [["WSO2", 700.0, 1], ["IBM", 70.0, 2], ["ORACLE", 75.0, 3], ["Aa", 1.0, 4], ["BB", 2.0, 5]]
case(name="partition_tie_hashmap_order", source="hand-traced: core/util/Scheduler.java:71-104,363-366, "
     "core/util/snapshot/state/PartitionStateHolder.java:36-83 (java.util.HashMap JDK 8)",
     schema="symbol string, price float, volume int",
     query=dict(window="time", param=1000, partition="symbol", aggs=[["sum", "price"]], output="all"),
     sends=[[[B] + r] for r in _tie] + [[[B + 1000 + i, f"x{i + 1}", 10.0 * (i + 1), 10 + i]] for i in range(5)],
     expect=dict(total_count=15,
                 values=[[700.0], [70.0], [75.0], [1.0], [2.0], [None], [10.0], [None], [20.0], [None], [30.0],
                         [None], [40.0], [None], [50.0]],
                 rep_cols=[["symbol", ["WSO2", "IBM", "ORACLE", "Aa", "BB", "BB", "x1", "Aa", "x2", "IBM", "x3",
                                       "WSO2", "x4", "ORACLE", "x5"]]]))

# partitioned lengthBatch(3) grouped by a column other than the partition key, `insert all events`,
# hand-traced (no reference test pins this shape; ctest/query/partition/WindowPartitionTestCase.java:96-139
# is the query form). Every completed batch of a partition is one chunk [previous batch EXPIRED, RESET,
# batch] (LengthBatchWindowProcessor.processFullBatchEvents :206-243) and processInBatchGroupBy
# (QuerySelector.java:315-374) keeps one row per side in first-insertion order (LinkedHashMap.put):
#   IBM batch 0 = buy 10, sell 20, buy 30   -> buy 40 (rep: buy 30), sell 20
#   WSO2 batch 0 = buy 1, sell 2, sell 3     -> buy 1, sell 5
#   IBM batch 1 = sell 5, sell 6, sell 7: chunk [EXPIRED buy 10, sell 20, buy 30, RESET, sell 5, 6, 7]:
#     buy first met as EXPIRED -> its last expired event with the state emptied (sum null);
#     sell first met as EXPIRED, then replaced by its last CURRENT row -> sell 18, at the EXPIRED position
case(name="partition_lengthBatch_group_by_other_all", source="hand-traced: core/query/selector/QuerySelector.java:315-374, "
     "core/query/processor/stream/window/LengthBatchWindowProcessor.java:206-243",
     schema="symbol string, side string, price int",
     query=dict(window="lengthBatch", param=3, partition="symbol", group_by=["side"], aggs=[["sum", "price"]],
                output="all"),
     sends=[[[B + i] + r] for i, r in enumerate([["IBM", "buy", 10], ["IBM", "sell", 20], ["WSO2", "buy", 1],
                                                ["IBM", "buy", 30], ["WSO2", "sell", 2], ["WSO2", "sell", 3],
                                                ["IBM", "sell", 5], ["IBM", "sell", 6], ["IBM", "sell", 7]])],
     expect=dict(total_count=6, values=[[40], [20], [1], [5], [None], [18]],
                 rep_cols=[["symbol", ["IBM", "IBM", "WSO2", "WSO2", "IBM", "IBM"]],
                           ["side", ["buy", "sell", "buy", "sell", "buy", "sell"]]]))

# ---------------------------------------------------------------- incremental aggregation (Aggregation1TestCase)
AGG_SCHEMA = "symbol string, price float, lastClosingPrice float, volume long, quantity int, timestamp long"
_t5 = [["WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["WSO2", 70.0, 0.0, 40, 10, 1496289950000],
       ["WSO2", 60.0, 44.0, 200, 56, 1496289952000], ["WSO2", 100.0, 0.0, 200, 16, 1496289952500],
       ["IBM", 100.0, 0.0, 200, 26, 1496289954000], ["IBM", 100.0, 0.0, 200, 96, 1496289954500]]
case(name="aggregation5_seconds", source="ctest/aggregation/Aggregation1TestCase.java:138-189",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "hour"]),
     sends=[[[r[-1]] + r] for r in _t5] + [{"advance": 1496289954500 + 3_600_000 * 2}],
     expect=dict(table="sec", rows=[[1496289952000, "WSO2", 80.0, 160.0], [1496289950000, "WSO2", 60.0, 120.0],
                                    [1496289954000, "IBM", 100.0, 200.0]]))
_t6 = [["WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["WSO2", 70.0, 0.0, 40, 10, 1496289950000],
       ["WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["WSO2", 70.0, 0.0, 40, 10, 1496289950000],
       ["IBM", 100.0, 0.0, 200, 26, 1496289951000], ["IBM", 100.0, 0.0, 200, 96, 1496289951000],
       ["IBM", 900.0, 0.0, 200, 60, 1496289952000], ["IBM", 500.0, 0.0, 200, 7, 1496289952000],
       ["WSO2", 60.0, 44.0, 200, 56, 1496289953000], ["WSO2", 100.0, 0.0, 200, 16, 1496289953000],
       ["IBM", 400.0, 0.0, 200, 9, 1496289953000], ["WSO2", 140.0, 0.0, 200, 11, 1496289953000],
       ["IBM", 600.0, 0.0, 200, 6, 1496289954000], ["IBM", 1000.0, 0.0, 200, 9, 1496290016000]]
case(name="aggregation6_seconds_to_year", source="ctest/aggregation/Aggregation1TestCase.java:191-299",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "year"]),
     sends=[[[r[-1]] + r] for r in _t6] + [{"advance": 1496290016000 + 400 * 86_400_000}],
     expect=dict(table="sec", rows=[[1496289950000, "WSO2", 60.0, 240.0], [1496289951000, "IBM", 100.0, 200.0],
                                    [1496289952000, "IBM", 700.0, 1400.0], [1496289953000, "WSO2", 100.0, 300.0],
                                    [1496289953000, "IBM", 400.0, 400.0], [1496289954000, "IBM", 600.0, 600.0],
                                    [1496290016000, "IBM", 1000.0, 1000.0]]))

# Retrieval KATs (`from A within ... per "<duration>"`) transcribed as the matching duration table:
# the tests' `within` ranges cover every bucket, and a TIMER past the last bucket (added here; the Java
# tests read the still-open buckets from the executors' in-memory state instead) moves every bucket
# into its table with the same base values (sums, counts are associative), so the table rows equal
# the retrieved rows. Columns the GPU does not aggregate (`price * quantity` as lastTradeValue) are
# not transcribed.
_t17 = [["WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["WSO2", 70.0, 0.0, 40, 10, 1496289950000],
        ["WSO2", 60.0, 44.0, 200, 56, 1496289952000], ["WSO2", 100.0, 0.0, 200, 16, 1496289952000],
        ["WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["WSO2", 70.0, 0.0, 40, 10, 1496289950000],
        ["IBM", 100.0, 0.0, 200, 26, 1496289954000], ["IBM", 100.0, 0.0, 200, 96, 1496289954000],
        ["IBM", 900.0, 0.0, 200, 60, 1496289956000], ["IBM", 500.0, 0.0, 200, 7, 1496289956000],
        ["IBM", 400.0, 0.0, 200, 9, 1496290016000], ["IBM", 600.0, 0.0, 200, 6, 1496290076000],
        ["CISCO", 700.0, 0.0, 200, 20, 1496293676000], ["WSO2", 60.0, 44.0, 200, 56, 1496297276000],
        ["CISCO", 800.0, 0.0, 100, 10, 1496383676000], ["CISCO", 900.0, 0.0, 100, 15, 1496470076000],
        ["IBM", 100.0, 0.0, 200, 96, 1499062076000], ["IBM", 400.0, 0.0, 200, 9, 1501740476000],
        ["WSO2", 60.0, 44.0, 200, 6, 1533276476000], ["WSO2", 260.0, 44.0, 200, 16, 1564812476000],
        ["CISCO", 260.0, 44.0, 200, 16, 1596434876000], ["CISCO", 260.0, 44.0, 200, 16, 1606975676000]]
_after_2020 = 1609459200000 + 400 * 86_400_000
case(name="aggregation17_months", source="ctest/aggregation/Aggregation1TestCase.java:704-839",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "year"]),
     sends=[[[r[-1]] + r] for r in _t17] + [{"advance": _after_2020}],
     expect=dict(table="month", rows=[[1496275200000, "WSO2", 65.71428571428571, 460.0],
                                      [1496275200000, "CISCO", 800.0, 2400.0],
                                      [1496275200000, "IBM", 433.3333333333333, 2600.0],
                                      [1498867200000, "IBM", 100.0, 100.0], [1501545600000, "IBM", 400.0, 400.0],
                                      [1533081600000, "WSO2", 60.0, 60.0], [1564617600000, "WSO2", 260.0, 260.0],
                                      [1596240000000, "CISCO", 260.0, 260.0], [1606780800000, "CISCO", 260.0, 260.0]]))
case(name="aggregation18_years", source="ctest/aggregation/Aggregation1TestCase.java:840-972",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "year"]),
     sends=[[[r[-1]] + r] for r in _t17] + [{"advance": _after_2020}],
     expect=dict(table="year", rows=[[1483228800000, "CISCO", 800.0, 2400.0], [1483228800000, "IBM", 387.5, 3100.0],
                                     [1483228800000, "WSO2", 65.71428571428571, 460.0],
                                     [1514764800000, "WSO2", 60.0, 60.0], [1546300800000, "WSO2", 260.0, 260.0],
                                     [1577836800000, "CISCO", 260.0, 520.0]]))
_t9 = [r for i, r in enumerate(_t17) if i not in (4, 5, 21)]  # test 9 sends each WSO2 pair once, no Dec 2020 event
case(name="aggregation9_days_no_group_by", source="ctest/aggregation/Aggregation1TestCase.java:300-428",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"], ["count", None]], group_by=[], ts="timestamp",
                      durations=["min", "year"]),
     sends=[[[r[-1]] + r] for r in _t9] + [{"advance": _after_2020}],
     expect=dict(table="day", rows=[[1496275200000, 303.3333333333333, 3640.0, 12], [1496361600000, 800.0, 800.0, 1],
                                    [1496448000000, 900.0, 900.0, 1], [1499040000000, 100.0, 100.0, 1],
                                    [1501718400000, 400.0, 400.0, 1], [1533254400000, 60.0, 60.0, 1],
                                    [1564790400000, 260.0, 260.0, 1], [1596412800000, 260.0, 260.0, 1]]))

# The same retrievals through the query path (sh_aggregation_find): no closing TIMER, so the
# latest buckets are read from the executors' in-memory stores as in the Java tests. `within` time
# strings are resolved to [start, end) here (the Java shim's job): "2017-01-01 00:00:00" (GMT) =
# 1483228800000, "2021-01-01 00:00:00" = 1609459200000, "2017-06-** **:**:**" = June 2017.
_jun2017 = [1496275200000, 1498867200000]
case(name="retrieval5_per_seconds", source="ctest/aggregation/Aggregation1TestCase.java:138-189",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "hour"]),
     sends=[[[r[-1]] + r] for r in _t5],
     expect=dict(find=dict(per="sec", start=_jun2017[0], end=_jun2017[1]),
                 rows=[[1496289952000, "WSO2", 80.0, 160.0], [1496289950000, "WSO2", 60.0, 120.0],
                       [1496289954000, "IBM", 100.0, 200.0]]))
case(name="retrieval9_per_days", source="ctest/aggregation/Aggregation1TestCase.java:300-428",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"], ["count", None]], group_by=[], ts="timestamp",
                      durations=["min", "year"]),
     sends=[[[r[-1]] + r] for r in _t9],
     expect=dict(find=dict(per="day", start=1496200000000, end=1596434876000),
                 rows=[[1496275200000, 303.3333333333333, 3640.0, 12], [1496361600000, 800.0, 800.0, 1],
                       [1496448000000, 900.0, 900.0, 1], [1499040000000, 100.0, 100.0, 1],
                       [1501718400000, 400.0, 400.0, 1], [1533254400000, 60.0, 60.0, 1],
                       [1564790400000, 260.0, 260.0, 1], [1596412800000, 260.0, 260.0, 1]]))
case(name="retrieval17_per_months", source="ctest/aggregation/Aggregation1TestCase.java:704-839",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "year"]),
     sends=[[[r[-1]] + r] for r in _t17],
     expect=dict(find=dict(per="month", start=1483228800000, end=1609459200000),
                 rows=[[1496275200000, "WSO2", 65.71428571428571, 460.0], [1496275200000, "CISCO", 800.0, 2400.0],
                       [1496275200000, "IBM", 433.3333333333333, 2600.0], [1498867200000, "IBM", 100.0, 100.0],
                       [1501545600000, "IBM", 400.0, 400.0], [1533081600000, "WSO2", 60.0, 60.0],
                       [1564617600000, "WSO2", 260.0, 260.0], [1596240000000, "CISCO", 260.0, 260.0],
                       [1606780800000, "CISCO", 260.0, 260.0]]))
case(name="retrieval18_per_years", source="ctest/aggregation/Aggregation1TestCase.java:840-972",
     kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["avg", "price"], ["sum", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "year"]),
     sends=[[[r[-1]] + r] for r in _t17],
     expect=dict(find=dict(per="year", start=1483228800000, end=1609459200000),
                 rows=[[1483228800000, "CISCO", 800.0, 2400.0], [1483228800000, "IBM", 387.5, 3100.0],
                       [1483228800000, "WSO2", 65.71428571428571, 460.0], [1514764800000, "WSO2", 60.0, 60.0],
                       [1546300800000, "WSO2", 260.0, 260.0], [1577836800000, "CISCO", 260.0, 520.0]]))

# ---------------------------------------------------------------- incremental aggregation (Aggregation2TestCase)
A2 = "ctest/aggregation/Aggregation2TestCase.java"
# tests 47 / 48 (no @app:playback: AGG_TIMESTAMP is the wall clock, the sends arrive within a few ms —
# modelled as send clocks B + i; `timestamp` carries the event time, out of order at the 4th send)
_t47 = [["WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["IBM", 100.0, 0.0, 200, 16, 1496289951011],
        ["IBM", 400.0, 0.0, 200, 9, 1496289952000], ["IBM", 900.0, 0.0, 200, 60, 1496289950000],
        ["WSO2", 500.0, 0.0, 200, 7, 1496289951011], ["IBM", 100.0, 0.0, 200, 26, 1496289953000],
        ["WSO2", 100.0, 0.0, 200, 96, 1496289953000]]
case(name="aggregation2_47_per_minutes", source=A2 + ":63-131", kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["sum", "price"], ["avg", "price"]], group_by=["symbol"], ts="timestamp",
                      durations=["sec", "year"]),
     sends=[[[B + i] + r] for i, r in enumerate(_t47)],
     expect=dict(find=dict(per="min", start=0, end=1543664151000),
                 rows=[[1496289900000, "WSO2", 650.0, 216.66666666666666], [1496289900000, "IBM", 1500.0, 375.0]]))
case(name="aggregation2_48_per_seconds", source=A2 + ":133-199", kind="aggregation", schema=AGG_SCHEMA,
     aggregation=dict(aggs=[["sum", "price"]], group_by=["symbol"], ts="timestamp", durations=["sec", "year"]),
     sends=[[[B + i] + r] for i, r in enumerate(_t47)],
     expect=dict(find=dict(per="sec", start=0, end=1543664151000),
                 rows=[[1496289950000, "WSO2", 50.0], [1496289950000, "IBM", 900.0], [1496289951000, "IBM", 100.0],
                       [1496289951000, "WSO2", 500.0], [1496289952000, "IBM", 400.0], [1496289953000, "IBM", 100.0],
                       [1496289953000, "WSO2", 100.0]]))
# aggTimeZone = Asia/Singapore (+08:00, no daylight saving): hour / day / month / year buckets start at
# Singapore's local boundaries (IncrementalTimeConverterUtil with the zone). `within "2019-**-** ..."`
# resolves in GMT (the Day5 / Year tables keep a bucket that starts at 16:00 GMT on Dec 31 of the year
# named): 2018 = [1514764800000, 1546300800000), 2019 = [.., 1577836800000), 2020 = [.., 1609459200000)
SGT = 8 * 3_600_000
_y = {2018: (1514764800000, 1546300800000), 2019: (1546300800000, 1577836800000),
      2020: (1577836800000, 1609459200000)}
_sgt = [  # (name, lines, root, year of `within`, the three event times, expected bucket starts)
    ("hour", "632-683", "hour", 2019, (1577721601000, 1577725199000, 1577725201000), (1577721600000, 1577725200000)),
    ("hour2", "685-737", "hour", 2020, (1582988401000, 1582991999000, 1582992001000), (1582988400000, 1582992000000)),
    ("day", "739-791", "day", 2020, (1580486401000, 1580572799000, 1580572801000), (1580486400000, 1580572800000)),
    ("day2", "793-845", "day", 2020, (1582905601000, 1582991999000, 1582992001000), (1582905600000, 1582992000000)),
    ("day3", "847-899", "day", 2019, (1551283201000, 1551369599000, 1551369601000), (1551283200000, 1551369600000)),
    ("day4", "901-953", "day", 2019, (1548864001000, 1548950399000, 1548950401000), (1548864000000, 1548950400000)),
    ("day5", "955-1007", "day", 2019, (1577721601000, 1577807999000, 1577808001000), (1577721600000, 1577808000000)),
    ("month", "1008-1060", "month", 2020, (1580486401000, 1582991999000, 1582992001000), (1580486400000, 1582992000000)),
]
for nm, lines, root, yr, ts3, b2 in _sgt:
    case(name=f"aggregation2_sgt_{nm}", source=f"{A2}:{lines}", kind="aggregation", schema="symbol string, price float, timestamp long",
         aggregation=dict(aggs=[["avg", "price"]], group_by=["symbol"], ts="timestamp", durations=[root, root],
                          tz_offset_ms=SGT),
         sends=[[[B + i, "WSO2", p, t]] for i, (p, t) in enumerate(zip((50.0, 70.0, 80.0), ts3))],
         expect=dict(find=dict(per=root, start=_y[yr][0], end=_y[yr][1]),
                     rows=[[b2[0], "WSO2", 60.0], [b2[1], "WSO2", 80.0]]))
case(name="aggregation2_sgt_year", source=A2 + ":1062-1115", kind="aggregation",
     schema="symbol string, price float, timestamp long",
     aggregation=dict(aggs=[["avg", "price"]], group_by=["symbol"], ts="timestamp", durations=["year", "year"],
                      tz_offset_ms=SGT),
     sends=[[[B + i, "WSO2", p, t]] for i, (p, t) in enumerate(zip((50.0, 70.0, 80.0),
                                                                 (1546272001000, 1577807999000, 1577808001000)))],
     expect=dict(find=dict(per="year", start=_y[2018][0], end=_y[2018][1]), rows=[[1546272000000, "WSO2", 60.0]]))

# SelectOptimisationAggregationTestCase.aggregationFunctionTestcase5: `group by symbol, name`, every sec, min;
# the reference joins the retrieval `within 1496200000000L, 1596434876000L per "seconds"` and sums count per
# symbol (WSO2 4, IBM 6, CISCO 1). The join is outside this path: the per-second rows below are hand-traced
# from the sends (two events per second bucket except the last three) and sum to those totals.
SO = "ctest/aggregation/SelectOptimisationAggregationTestCase.java"
_so5 = [["WSO2", "WSO2", 50.0, 60.0, 90, 6, 1496289950000], ["WSO2", "WSO2", 70.0, 0.0, 40, 10, 1496289950000],
        ["WSO2", "WSO2", 60.0, 44.0, 200, 56, 1496289952000], ["WSO2", "WSO2", 100.0, 0.0, 200, 16, 1496289952000],
        ["IBM", "IBM", 100.0, 0.0, 200, 26, 1496289954000], ["IBM", "IBM", 100.0, 0.0, 200, 96, 1496289954000],
        ["IBM", "IBM", 900.0, 0.0, 200, 60, 1496289956000], ["IBM", "IBM", 500.0, 0.0, 200, 7, 1496289956000],
        ["IBM", "IBM", 400.0, 0.0, 200, 9, 1496290016000], ["IBM", "IBM", 600.0, 0.0, 200, 6, 1496290076000],
        ["CISCO", "CISCO", 700.0, 0.0, 200, 20, 1496293676000]]
case(name="select_optimisation5_two_group_by", source=SO + ":436-525", kind="aggregation",
     schema="symbol string, name string, price float, lastClosingPrice float, volume long, quantity int, timestamp long",
     aggregation=dict(aggs=[["count", None]], group_by=["symbol", "name"], ts="timestamp", durations=["sec", "min"]),
     sends=[[[B + i] + r] for i, r in enumerate(_so5)],
     expect=dict(find=dict(per="sec", start=1496200000000, end=1596434876000),
                 rows=[[1496289950000, "WSO2", "WSO2", 2], [1496289952000, "WSO2", "WSO2", 2],
                       [1496289954000, "IBM", "IBM", 2], [1496289956000, "IBM", "IBM", 2],
                       [1496290016000, "IBM", "IBM", 1], [1496290076000, "IBM", "IBM", 1],
                       [1496293676000, "CISCO", "CISCO", 1]]))

# ---------------------------------------------------------------- filters (FilterTestCase1): expected counts
F = "ctest/query/FilterTestCase1.java"
FL = "symbol string, price float, volume long"
case(name="filter1", source=F + ":60-118", schema=FL, query=dict(window=None, filter=[">", 70, "price"]),
     sends=[[[B, "IBM", 700.0, 100]], [[B + 1, "WSO2", 60.5, 200]]], expect=dict(in_count=1))
case(name="filter2", source=F + ":120-152", schema=FL, query=dict(window=None, filter=[">", 150, "volume"]),
     sends=[[[B, "IBM", 700.0, 100]], [[B + 1, "WSO2", 60.5, 200]]], expect=dict(in_count=1))
case(name="filter3", source=F + ":154-186", schema=CSE_FLOAT_INT, query=dict(window=None, filter=[">", 70, "price"]),
     sends=[[[B, "WSO2", 55.6, 100]], [[B + 1, "IBM", 75.6, 100]], [[B + 2, "WSO2", 57.6, 200]]],
     expect=dict(in_count=2))
_v3 = lambda schema_t: [[[B, "WSO2", 50.0, 60]], [[B + 1, "WSO2", 70.0, 40]], [[B + 2, "WSO2", 44.0, 200]]]
for nm, rng, vt, const in [("filter4", ":188-217", "long", ["float", 50.0]), ("filter5", ":219-249", "long", ["long", 50]),
                           ("filter6", ":251-281", "int", ["long", 50]), ("filter7", ":283-313", "double", ["long", 50]),
                           ("filter8", ":315-346", "float", ["long", 50]), ("filter9", ":348-379", "float", ["float", 50.0]),
                           ("filter10", ":381-411", "double", ["double", 50.0]),
                           ("filter11", ":413-443", "double", ["float", 50.0]),
                           ("filter12", ":445-475", "double", ["int", 45]),
                           ("filter13", ":477-507", "float", ["double", 50.0]),
                           ("filter14", ":509-539", "float", ["int", 45]),
                           ("filter16", ":574-603", "long", ["double", 50.0])]:
    case(name=nm, source=F + rng, schema=f"symbol string, price float, volume {vt}",
         query=dict(window=None, filter=[">", "volume", const]), sends=_v3(vt), expect=dict(in_count=2))
case(name="filter15", source=F + ":541-572", schema="symbol string, price float, volume float, quantity int",
     query=dict(window=None, filter=[">", "quantity", ["double", 4.0]]),
     sends=[[[B, "WSO2", 50.0, 60.0, 5]], [[B + 1, "WSO2", 70.0, 60.0, 2]], [[B + 2, "WSO2", 60.0, 200.0, 4]]],
     expect=dict(in_count=1))
case(name="filter21", source=F + ":746-776", schema=FL, query=dict(window=None, filter=["!=", "volume", 100]),
     sends=[[[B, "WSO2", 55.6, 100]], [[B + 1, "WSO2", 57.6, 10]]], expect=dict(in_count=1))
case(name="filter22", source=F + ":778-810", schema="symbol string, price float, volume double",
     query=dict(window=None, filter=["and", [">", "volume", ["long", 12]], ["<", "price", 56]]),
     sends=[[[B, "WSO2", 55.6, 100.0]], [[B + 1, "WSO2", 57.6, 10.0]]], expect=dict(in_count=1))
case(name="filter23", source=F + ":812-841", schema=FL,
     query=dict(window=None, filter=["and", ["and", ["!=", "symbol", ["string", "WSO2"]], ["!=", "volume", ["long", 55]]],
                                     ["!=", "price", ["float", 45.0]]]),
     sends=[[[B, "WSO2", 45.0, 100]], [[B + 1, "IBM", 35.0, 50]]], expect=dict(in_count=1))
case(name="filter24", source=F + ":843-873", schema=FL, query=dict(window=None, filter=["!=", "volume", ["float", 50.0]]),
     sends=[[[B, "WSO2", 45.0, 100]], [[B + 1, "IBM", 35.0, 50]]], expect=dict(in_count=1))
case(name="filter25", source=F + ":875-906", schema=FL, query=dict(window=None, filter=["!=", "price", ["long", 35]]),
     sends=[[[B, "WSO2", 45.0, 100]], [[B + 1, "IBM", 35.0, 50]]], expect=dict(in_count=1))
case(name="filter26", source=F + ":908-938", schema=FL,
     query=dict(window=None, filter=["and", ["!=", "volume", 100], ["!=", "volume", ["double", 70.0]]]),
     sends=[[[B, "WSO2", 55.6, 100]], [[B + 1, "IBM", 57.6, 10]]], expect=dict(in_count=1))
case(name="filter27", source=F + ":940-969", schema=FL,
     query=dict(window=None, filter=["or", ["!=", "price", ["double", 53.6]], ["!=", "price", 87]]),
     sends=[[[B, "WSO2", 55.6, 100]], [[B + 1, "IBM", 57.6, 10]]], expect=dict(in_count=2))
case(name="filter28", source=F + ":971-1002", schema=CSE_FLOAT_INT,
     query=dict(window=None, filter=["and", ["!=", "volume", ["float", 40.0]], ["!=", "volume", 400]]),
     sends=[[[B, "WSO2", 55.5, 40]], [[B + 1, "WSO2", 53.5, 50]], [[B + 2, "WSO2", 50.5, 400]]],
     expect=dict(in_count=1))
case(name="filter29", source=F + ":1004-1034", schema=CSE_FLOAT_INT,
     query=dict(window=None, filter=["and", ["!=", "volume", ["double", 40.0]], ["!=", "volume", ["double", 400.0]]]),
     sends=[[[B, "WSO2", 55.5, 40]], [[B + 1, "WSO2", 53.5, 50]], [[B + 2, "WSO2", 50.5, 400]]],
     expect=dict(in_count=1))
case(name="filter30_bool", source=F + ":1036-1064", schema="symbol string, price float, available bool",
     query=dict(window=None, filter=["!=", "available", ["bool", 1]]),
     sends=[[[B, "IBM", 55.6, True]], [[B + 1, "WSO2", 57.6, False]]], expect=dict(in_count=1))

# ------------------------------------------------- output rate limiting (EventOutputRateLimitTestCase)
# `output [all|first|last] every N events` over the selector's rows (OutputParser.java:288-303). The
# Java tests send one event per InputHandler.send (each send is one chunk for the limiter).
R = "ctest/query/ratelimit/EventOutputRateLimitTestCase.java"


def _ips(*ips):
    return [[[B + i, B + i, "192.10.1." + str(x)]] for i, x in enumerate(ips)]


def _ip(*xs):
    return ["192.10.1." + str(x) for x in xs]


case(name="rate1_all2", source=R + ":45-97", schema=LOGIN, query=dict(window=None, rate=["all", 2]),
     sends=_ips(3, 3, 4, 3, 5), expect=dict(in_count=4, remove_count=0))
case(name="rate2_default_all2", source=R + ":99-149", schema=LOGIN, query=dict(window=None, rate=["all", 2]),
     sends=_ips(3, 3, 4, 3, 5), expect=dict(in_count=4, remove_count=0))
case(name="rate3_all5", source=R + ":151-205", schema=LOGIN, query=dict(window=None, rate=["all", 5]),
     sends=_ips(5, 5, 3, 9, 4, 4, 4, 30), expect=dict(in_count=5, remove_count=0))
case(name="rate4_first2", source=R + ":207-260", schema=LOGIN, query=dict(window=None, rate=["first", 2]),
     sends=_ips(5, 3, 9, 4, 3), expect=dict(in_count=3, remove_count=0, in_col_in=["ip", _ip(5, 9, 3)]))
case(name="rate5_first3", source=R + ":262-314", schema=LOGIN, query=dict(window=None, rate=["first", 3]),
     sends=_ips(5, 3, 9, 4, 3), expect=dict(in_count=2, remove_count=0, in_col_in=["ip", _ip(5, 4)]))
case(name="rate6_last2", source=R + ":316-368", schema=LOGIN, query=dict(window=None, rate=["last", 2]),
     sends=_ips(3, 5, 3, 4, 3), expect=dict(in_count=2, remove_count=0, in_col_in=["ip", _ip(5, 4)]))
case(name="rate7_last4", source=R + ":370-421", schema=LOGIN, query=dict(window=None, rate=["last", 4]),
     sends=_ips(3, 5, 3, 4, 3), expect=dict(in_count=1, remove_count=0, in_col_in=["ip", _ip(4)]))
case(name="rate8_first5_group_by", source=R + ":423-476", schema=LOGIN,
     query=dict(window=None, group_by=["ip"], rate=["first", 5]),
     sends=_ips(5, 5, 3, 9, 4, 4, 4, 30), expect=dict(in_count=5, remove_count=0))
case(name="rate9_last5_group_by", source=R + ":478-533", schema=LOGIN,
     query=dict(window=None, group_by=["ip"], rate=["last", 5]),
     sends=_ips(5, 5, 3, 9, 4, 4, 4, 30), expect=dict(in_count=4, remove_count=0))
case(name="rate10_first5_group_by", source=R + ":535-590", schema=LOGIN,
     query=dict(window=None, group_by=["ip"], rate=["first", 5]),
     sends=_ips(5, 5, 3, 9, 4, 4, 4, 4, 4, 30), expect=dict(in_count=5, remove_count=0))
case(name="rate11_last5_group_by", source=R + ":592-649", schema=LOGIN,
     query=dict(window=None, group_by=["ip"], rate=["last", 5]),
     sends=_ips(5, 5, 3, 9, 4, 4, 4, 30, 3, 30), expect=dict(in_count=7, remove_count=0))
_r12 = _ips(5, 3, 3, 9, 3, 4, 4, 4, 30, 31, 32, 33)
case(name="rate12_lengthBatch_last5_group_by", source=R + ":651-710", schema=LOGIN,
     query=dict(window="lengthBatch", param=4, group_by=["ip"], aggs=[["count", None]], rate=["last", 5]),
     sends=_r12, expect=dict(in_count=4, remove_count=0))
case(name="rate13_lengthBatch_last2", source=R + ":712-769", schema=LOGIN,
     query=dict(window="lengthBatch", param=4, aggs=[["count", None]], rate=["last", 2]),
     sends=_r12, expect=dict(in_count=1, remove_count=0))
case(name="rate14_lengthBatch_expired_last2", source=R + ":771-829", schema=LOGIN,
     query=dict(window="lengthBatch", param=4, aggs=[["count", None]], output="expired", rate=["last", 2]),
     sends=_r12, expect=dict(in_count=0, remove_count=1))
case(name="rate15_lengthBatch_expired_all2", source=R + ":831-888", schema=LOGIN,
     query=dict(window="lengthBatch", param=4, aggs=[["count", None]], output="expired", rate=["all", 2]),
     sends=_r12, expect=dict(in_count=0, remove_count=2))
case(name="rate16_lengthBatch_expired_all2_group_by", source=R + ":890-948", schema=LOGIN,
     query=dict(window="lengthBatch", param=4, group_by=["ip"], aggs=[["count", None]], output="expired",
                rate=["all", 2]),
     sends=_r12, expect=dict(in_count=0, remove_count=4))
case(name="rate17_first2_group_by", source=R + ":950-1006", schema=LOGIN,
     query=dict(window=None, group_by=["ip"], rate=["first", 2]),
     sends=_ips(5, 5, 3, 5, 5, 9, 4, 4, 4, 5, 30), expect=dict(in_count=8, remove_count=0))
case(name="rate18_first2", source=R + ":1008-1066", schema=LOGIN, query=dict(window=None, rate=["first", 2]),
     sends=_ips(5, 3, 5, 5, 5, 9, 4, 4, 4, 30, 5),
     expect=dict(in_count=6, remove_count=0, in_col_in=["ip", _ip(5, 4)]))

# `output first every 1 sec` (TimeOutputRateLimitTestCase): FirstPerTime / FirstGroupByPerTime read the
# TimestampGenerator, so in playback the clock of each send decides; the Java tests' sends land at
# t, t (+ ms), then 1100 ms later, then 2200 ms later (Thread.sleep between them).
T_ = "ctest/query/ratelimit/TimeOutputRateLimitTestCase.java"


def _tips(*pairs):
    return [[[B + dt, B + dt, "192.10.1." + str(x)]] for dt, x in pairs]


case(name="trate4_first_every_1s", source=T_ + ":223-280", schema=LOGIN,
     query=dict(window=None, rate=["first_time", 1000]),
     sends=_tips((0, 5), (0, 3), (1100, 9), (1100, 4), (2200, 30)),
     expect=dict(in_count=3, remove_count=0, in_col_in=["ip", _ip(5, 9, 30)]))
case(name="trate6_first_every_1s_group_by", source=T_ + ":341-398", schema=LOGIN,
     query=dict(window=None, group_by=["ip"], rate=["first_time", 1000]),
     sends=_tips((0, 5), (0, 5), (0, 3), (0, 9), (0, 4), (1100, 4), (1100, 4), (1100, 30)),
     expect=dict(in_count=6, remove_count=0))

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_reference.json")
    with open(out, "w") as f:
        json.dump({"generated_by": "tests/golden/make_kat.py", "cases": CASES}, f, indent=1)
    print(f"wrote {len(CASES)} cases to {out}")
