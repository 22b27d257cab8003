"""Writes tests/golden/reference_cases.json: the inputs and asserted outcomes of
the reference's own unit tests for the block codec, transcribed as DATA (no
reference source text): item lists, restart intervals, hash ratios, and what
each Rust assert says the result must be.  Expected outcomes are hard-coded from
the asserts, not computed by the oracle, so they pin the oracle and the GPU to
the reference itself.

Sources (fjall-rs/lsm-tree 3.1.9):
  src/table/data_block/mod.rs:565-1235     DataBlock point_read / len / index tests
  src/table/data_block/iter_test.rs:13-1280  iterator, seek, seek_upper, range tests
  src/table/index_block/iter.rs:68-672     index block round trips (forward parts)
  src/table/block/hash_index/mod.rs:48-142 hash index bytes / conflicts
  src/table/block/header.rs:177-214        header round trip / corruption

Item = [key hex, value hex, seqno, vtype] (vtype 0 Value, 1 Tombstone, 4 Indirection).
Point read = [needle hex, snapshot seqno, expected item index or None, is_tombstone or None].
Range = {"lo", "hi": bound hex or None, "lo_found", "hi_found": seek/seek_upper return
values (None = not asserted), "range": [first, end) item indexes every iteration order
(next, next_back, ping-pong) yields}.  SeqNo::MAX = 2^64 - 1.

Run: python tests/golden/make_reference_cases.py
"""
import json
from pathlib import Path

MAX = (1 << 64) - 1
V, T, I = 0, 1, 4


def h(b):
    return bytes(b).hex() if not isinstance(b, str) else b.encode().hex()


def it(k, v, s, t):
    return [h(k), h(v), s, t]


def be(i):
    return list(i.to_bytes(8, "big"))


RI16 = list(range(1, 17))
BCDEF = [it("b", "b", 0, V), it("c", "c", 0, V), it("d", "d", 1, T), it("e", "e", 0, V), it("f", "f", 0, V)]
PLA5 = [it("pla:earth:fact", "eaaaaaaaaarth", 0, V), it("pla:jupiter:fact", "Jupiter is big", 0, V),
        it("pla:jupiter:mass", "Massive", 0, V), it("pla:jupiter:name", "Jupiter", 0, V),
        it("pla:jupiter:radius", "Big", 0, V)]
MVCC_LATEST = [it([0], [], 0, V)] + [it([233, 233], [], s, V) for s in range(8, -1, -1)] + \
              [it([255, 255, 0], [], 127_886_946_205_696, T)]


def each_item_reads(items, snap_plus_one=True):
    return [[k, (s + 1) if snap_plus_one else MAX, i, None] for i, (k, _, s, _) in enumerate(items)]


def rng(lo=None, hi=None, first=0, end=0, lo_found=None, hi_found=None):
    return {"lo": lo, "hi": hi, "lo_found": lo_found, "hi_found": hi_found, "range": [first, end]}


data_block = []


def case(name, ref, items, ris, ratio, **expect):
    data_block.append({"name": name, "ref": ref, "items": items, "restart_intervals": ris, "hash_ratio": ratio,
                       "expect": expect})


# ---- src/table/data_block/mod.rs
case("data_block_ping_pong_fuzz_1", "src/table/data_block/mod.rs:565-632",
     [it([111], [119], 8_602_264_972_526_186_597, V), it([121, 120, 99], [101] * 11, 11_426_548_769_907, V)],
     [1], 0.0, forward=True, ranges=[rng(first=0, end=2)])
case("data_block_point_read_simple", "src/table/data_block/mod.rs:634-674", BCDEF, RI16, 0.0,
     point_reads=[[h("a"), MAX, None, None], [h("b"), MAX, 0, None], [h("z"), MAX, None, None]])
case("data_block_point_read_one", "src/table/data_block/mod.rs:676-712",
     [it("pla:earth:fact", "eaaaaaaaaarth", 0, V)], [16], 0.0, len=1, binary_index_len=1,
     point_reads=[[h("pla:earth:fact"), MAX, 0, None], [h("yyy"), MAX, None, None]])
case("data_block_vhandle", "src/table/data_block/mod.rs:714-745", [it("abc", "world", 1, I)], RI16, 0.0, len=1,
     point_reads=[[h("abc"), 777, 0, None], [h("abc"), 1, None, None]])
case("data_block_mvcc_read_first", "src/table/data_block/mod.rs:747-777", [it("hello", "world", 0, V)], RI16, 0.0,
     len=1, point_reads=[[h("hello"), 777, 0, None]])
items = [it([0], [], 23_523_531_241_241_242, V), it([0], [], 0, V)]
case("data_block_point_read_fuzz_1", "src/table/data_block/mod.rs:779-816", items, [16], 1.33, len=2,
     hash_index=True, point_reads=each_item_reads(items) + [[h("yyy"), MAX, None, None]])
items = [it([0], [], 5, V), it([0], [], 4, T), it([0], [], 3, V), it([0], [], 0, V)]
case("data_block_point_read_fuzz_2", "src/table/data_block/mod.rs:818-852", items, [2], 0.0, len=4,
     hash_index=False, point_reads=each_item_reads(items) + [[h("yyy"), MAX, None, None]])
items = [it("a", "a", 3, V), it("b", "b", 2, V), it("c", "c", 1, V), it("d", "d", 65, V)]
case("data_block_point_read_dense", "src/table/data_block/mod.rs:854-888", items, [1], 0.0, len=4,
     binary_index_len=4, point_reads=each_item_reads(items, False) + [[h("yyy"), MAX, None, None]])
items = [it("a", "a", 3, V), it("a", "a", 2, V), it("a", "a", 1, V), it("b", "b", 65, V)]
case("data_block_point_read_dense_mvcc_with_hash", "src/table/data_block/mod.rs:890-929", items, [1], 1.33, len=4,
     hash_index=True, point_reads=each_item_reads(items) + [[h("yyy"), MAX, None, None]])
case("data_block_point_read_mvcc_latest_fuzz_1", "src/table/data_block/mod.rs:931-967",
     [it([0], [], 0, V), it([233, 233], [], 0, V), it([255, 255, 0], [], 127_886_946_205_696, T)], [2], 0.0,
     len=3, hash_index=False, point_reads=[[h([233, 233]), MAX, 1, None], [h("yyy"), MAX, None, None]])
for nm, ref, ri in (("data_block_point_read_mvcc_latest_fuzz_2", "src/table/data_block/mod.rs:969-1016", 2),
                    ("data_block_point_read_mvcc_latest_fuzz_3", "src/table/data_block/mod.rs:1018-1065", 2),
                    ("data_block_point_read_mvcc_latest_fuzz_3_dense", "src/table/data_block/mod.rs:1067-1114", 1)):
    case(nm, ref, MVCC_LATEST, [ri], 0.0, len=11,
         point_reads=[[h([233, 233]), MAX, 1, None], [h([255, 255, 0]), MAX, 10, True], [h("yyy"), MAX, None, None]])
items = [it("a", "a", 3, V), it("a", "a", 2, V), it("a", "a", 1, V), it("b", "b", 65, V)]
case("data_block_point_read_dense_mvcc_no_hash", "src/table/data_block/mod.rs:1116-1150", items, [1], 0.0, len=4,
     hash_index=False, point_reads=each_item_reads(items) + [[h("yyy"), MAX, None, None]])
case("data_block_point_read_shadowing", "src/table/data_block/mod.rs:1152-1188",
     [it("pla:saturn:fact", "Saturn is pretty big", 0, V), it("pla:saturn:name", "Saturn", 0, V),
      it("pla:venus:fact", "", 1, T), it("pla:venus:fact", "Venus exists", 0, V), it("pla:venus:name", "Venus", 0, V)],
     [16], 1.33, len=5, hash_index=True, point_reads=[[h("pla:venus:fact"), MAX, 2, True]])
items = [it("pla:earth:fact", "eaaaaaaaaarth", 0, V), it("pla:jupiter:fact", "Jupiter is big", 0, V),
         it("pla:jupiter:mass", "Massive", 0, V), it("pla:jupiter:name", "Jupiter", 0, V),
         it("pla:jupiter:radius", "Big", 0, V), it("pla:saturn:fact", "Saturn is pretty big", 0, V),
         it("pla:saturn:name", "Saturn", 0, V), it("pla:venus:fact", "", 1, T), it("pla:venus:fact", "Venus exists", 0, V),
         it("pla:venus:name", "Venus", 0, V)]
case("data_block_point_read_dense_2", "src/table/data_block/mod.rs:1190-1235", items, [1], 1.33, len=10,
     hash_index=True, point_reads=each_item_reads(items) + [[h("yyy"), MAX, None, None]])

# ---- src/table/data_block/iter_test.rs
items = [it(be(i), "", 0, V) for i in range(108, 144)]
case("data_block_wtf", "src/table/data_block/iter_test.rs:13-125", items, RI16, 1.33,
     ranges=[rng(h(be(10)), h(be(110)), 0, 3)])
items = [it(be(i), "", 0, V) for i in range(100, 110)]
case("data_block_range", "src/table/data_block/iter_test.rs:127-199", items, RI16, 1.33,
     ranges=[rng(h(be(10)), h(be(109)), 0, 10)])
items = [it(be(i), "", 0, V) for i in range(0, 100)]
case("data_block_range_ping_pong", "src/table/data_block/iter_test.rs:201-247", items, RI16, 1.33,
     ranges=[rng(h(be(5)), h(be(9)), 5, 10)])
case("data_block_iter_forward", "src/table/data_block/iter_test.rs:249-282", BCDEF, RI16, 1.33, forward=True)
case("data_block_iter_rev", "src/table/data_block/iter_test.rs:284-321", BCDEF, RI16, 1.33, forward=True,
     ranges=[rng(first=0, end=5)])
case("data_block_iter_rev_seek_back", "src/table/data_block/iter_test.rs:323-361", BCDEF, RI16, 0.0,
     ranges=[rng(hi=h("d"), hi_found=True, first=0, end=3)])
case("data_block_iter_range_edges", "src/table/data_block/iter_test.rs:363-442", BCDEF, RI16, 0.0,
     ranges=[rng(lo=h("a"), lo_found=False, first=0, end=5), rng(hi=h("g"), hi_found=False, first=0, end=5),
             rng(hi=h("b"), hi_found=True, first=0, end=1), rng(lo=h("f"), lo_found=True, first=4, end=5)])
case("data_block_iter_range", "src/table/data_block/iter_test.rs:444-483", BCDEF, RI16, 0.0,
     ranges=[rng(h("c"), h("d"), 1, 3, True, True)])
case("data_block_iter_only_first", "src/table/data_block/iter_test.rs:485-523", BCDEF, RI16, 0.0,
     ranges=[rng(hi=h("b"), hi_found=True, first=0, end=1)])
case("data_block_iter_range_same_key", "src/table/data_block/iter_test.rs:525-626", BCDEF, RI16, 0.0,
     ranges=[rng(h("d"), h("d"), 2, 3, True, True)])
case("data_block_iter_range_empty", "src/table/data_block/iter_test.rs:628-697", BCDEF, RI16, 0.0,
     ranges=[rng(h("f"), h("e"), 4, 4, True, True)])
case("data_block_iter_forward_seek_restart_head", "src/table/data_block/iter_test.rs:699-734", BCDEF, RI16, 1.33,
     ranges=[rng(lo=h("b"), lo_found=True, first=0, end=5)])
case("data_block_iter_forward_seek_in_interval", "src/table/data_block/iter_test.rs:736-774", BCDEF, RI16, 1.33,
     ranges=[rng(lo=h("d"), lo_found=True, first=2, end=5)])
case("data_block_iter_forward_seek_last", "src/table/data_block/iter_test.rs:776-814", BCDEF, RI16, 1.33,
     ranges=[rng(lo=h("f"), lo_found=True, first=4, end=5)])
case("data_block_iter_forward_seek_before_first", "src/table/data_block/iter_test.rs:816-851", BCDEF, RI16, 1.33,
     ranges=[rng(lo=h("a"), lo_found=False, first=0, end=5)])
case("data_block_iter_forward_seek_after_last", "src/table/data_block/iter_test.rs:853-884", BCDEF, RI16, 1.33,
     ranges=[rng(lo=h("g"), lo_found=False, first=5, end=5)])
case("data_block_iter_consume_last_back", "src/table/data_block/iter_test.rs:886-972", PLA5, RI16, 0.0, len=5,
     hash_index=False, forward=True, ranges=[rng(first=0, end=5)])
case("data_block_iter_consume_last_forwards", "src/table/data_block/iter_test.rs:974-1062", PLA5, RI16, 0.0, len=5,
     hash_index=False, forward=True, ranges=[rng(first=0, end=5)])
case("data_block_iter_ping_pong_exhaust", "src/table/data_block/iter_test.rs:1064-1152",
     [it(c, c, 0, V) for c in "abcde"], list(range(1, 256)), 0.0, len=5, hash_index=False, forward=True,
     ranges=[rng(first=0, end=5)])
case("data_block_iter_fuzz_3", "src/table/data_block/iter_test.rs:1154-1197",
     [it([255, 255, 255, 255, 5] + [255] * 16, [0, 0, 192], 18_446_744_073_701_163_007, T),
      it([255, 255, 255, 255, 255, 255, 0], [], 0, V)], [5], 1.0, len=2, hash_index=True, count=2)
case("data_block_iter_fuzz_4", "src/table/data_block/iter_test.rs:1199-1247",
     [it([0], [], 3_834_029_160_418_063_669, V), it([0], [], 127, T), it([53, 53, 53], [], MAX, T),
      it([255], [], 18_446_744_069_414_584_831, T), it([255, 255], [], 47, V)], [2], 1.0, len=5, hash_index=True,
     count=5)
case("data_block_seek_closed_range", "src/table/data_block/iter_test.rs:1249-1279",
     [it([0, 161], [], 1, T), it([0, 161], [], 0, T), it([1], [], 0, V)], [100], 0.0, len=3, count=3,
     ranges=[rng(h([0]), h([0]), 0, 0)])

# ---- src/table/index_block/iter.rs (KeyedBlockHandle = end key, seqno, offset, size)
B3 = [[h("b"), 0, 0, 6000], [h("bcdef"), 0, 6000, 7000], [h("def"), 0, 13000, 5000]]
index_block = [
    {"name": n, "ref": "src/table/index_block/iter.rs:" + r, "items": B3, "expect": {"len": 3, "forward": True}}
    for n, r in (("index_block_iter_seek_before_start", "68-110"), ("index_block_iter_seek_start", "112-152"),
                 ("index_block_iter_seek_middle", "154-197"), ("index_block_iter_rev_seek", "199-239"),
                 ("index_block_iter_rev_seek_2", "241-281"), ("index_block_iter_rev_seek_3", "283-326"),
                 ("index_block_iter_too_far", "328-368"), ("index_block_iter_too_far_next_back", "370-408"))]
index_block += [
    {"name": "index_block_mvcc_slab", "ref": "src/table/index_block/iter.rs:410-511",
     "items": [[h("a"), 3, 0, 6000], [h("a"), 1, 6000, 7000], [h("b"), 4, 13000, 5000]],
     "expect": {"len": 3, "forward": True}},
    {"name": "index_block_iter_span", "ref": "src/table/index_block/iter.rs:513-561",
     "items": [[h("a"), 1, 0, 6000], [h("a"), 0, 6000, 7000], [h("b"), 0, 13000, 5000]],
     "expect": {"len": 3, "forward": True}},
    {"name": "index_block_iter_rev_span", "ref": "src/table/index_block/iter.rs:563-608",
     "items": [[h("a"), 1, 0, 6000], [h("a"), 0, 6000, 7000], [h("b"), 0, 13000, 5000]],
     "expect": {"len": 3, "forward": True}},
    {"name": "index_block_iter_range_1", "ref": "src/table/index_block/iter.rs:610-671",
     "items": [[h("a"), 0, 0, 6000]] + [[h(c), 0, 13000, 5000] for c in "bcde"],
     "expect": {"len": 5, "forward": True}},
]

# ---- src/table/block/hash_index/mod.rs (bucket byte 254 = FREE, 255 = CONFLICT)
simple = [254] * 100
simple[11], simple[15], simple[19] = 10, 8, 5
hash_index = [
    {"name": "hash_index_build_simple", "ref": "src/table/block/hash_index/mod.rs:48-79", "buckets": 100,
     "sets": [[h("a"), 5], [h("b"), 8], [h("c"), 10]], "bytes": simple, "conflicts": 0,
     "gets": [[h("a"), 5], [h("b"), 8], [h("c"), 10], [h("d"), 254]]},
    {"name": "hash_index_build_conflict", "ref": "src/table/block/hash_index/mod.rs:81-93", "buckets": 1,
     "sets": [[h("a"), 5], [h("b"), 8]], "bytes": [255], "conflicts": 1, "gets": []},
    {"name": "hash_index_build_same_offset", "ref": "src/table/block/hash_index/mod.rs:95-110", "buckets": 1,
     "sets": [[h("a"), 5], [h("b"), 5]], "bytes": [5], "conflicts": 0, "gets": [[h("a"), 5], [h("b"), 5]]},
    {"name": "hash_index_build_mix", "ref": "src/table/block/hash_index/mod.rs:112-125", "buckets": 1,
     "sets": [[h("a"), 5], [h("b"), 5], [h("c"), 6]], "bytes": [255], "conflicts": 1, "gets": []},
    {"name": "hash_index_read_conflict", "ref": "src/table/block/hash_index/mod.rs:127-142", "buckets": 1,
     "sets": [[h("a"), 5], [h("b"), 8]], "bytes": [255], "conflicts": 1,
     "gets": [[h("a"), 255], [h("b"), 255], [h("c"), 255]]},
]

# ---- src/table/block/header.rs (checksum = Checksum::from_raw(5): the 128-bit field holds 5)
header = [
    {"name": "block_header_serde_roundtrip", "ref": "src/table/block/header.rs:177-192",
     "block_type": 0, "checksum": 5, "data_length": 252_356, "uncompressed_length": 124_124_124,
     "mutate_byte": None, "expect": "OK"},
    {"name": "block_header_detect_corruption", "ref": "src/table/block/header.rs:194-214",
     "block_type": 0, "checksum": 5, "data_length": 252_356, "uncompressed_length": 124_124_124,
     "mutate_byte": 5, "expect": "HDR_CKSUM"},
]

out = {"source": "fjall-rs/lsm-tree 3.1.9 unit tests: inputs and asserted outcomes transcribed as data",
       "data_block": data_block, "index_block": index_block, "hash_index": hash_index, "header": header}
Path(__file__).with_name("reference_cases.json").write_text(json.dumps(out, indent=1) + "\n")
print(f"{len(data_block)} data block, {len(index_block)} index block, {len(hash_index)} hash index, "
      f"{len(header)} header cases")
