"""Writes tests/golden/kats.json: known-answer tests for the RWI hot path.

Inputs are hand-built 40-byte WordReferenceRow rows; every expected value is
written out here by hand -- derived from the reference's own JUnit assertions
or by reading the cited reference lines -- and is NOT computed by the oracle.
Run:  python tests/golden/make_kats.py
"""

import json
import os

ALPHA = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
DAY = 86400000


def row(h, a=15000, s=0, u=2, w=15, p=3, d="t", l="en", x=0, y=0, m=25, n=3, g=0, z=0,
        c=1, t=1, r=1, o=100, i=0, k=0):
    """Encode a 40-byte WordReferenceRow (WordReferenceRow.java:49-72)."""
    assert len(h) == 12 and all(ch in ALPHA for ch in h)
    b = bytearray(40)
    b[0:12] = h.encode()
    b[12:14] = a.to_bytes(2, "big")
    b[14:16] = s.to_bytes(2, "big")
    b[16] = u
    b[17:19] = w.to_bytes(2, "big")
    b[19:21] = p.to_bytes(2, "big")
    b[21] = ord(d)
    b[22:24] = l.encode() if l else b"\x00\x00"
    b[24], b[25], b[26], b[27], b[28] = x, y, m, n, g
    b[29:33] = z.to_bytes(4, "little")  # Bitfield: bit b in byte b>>3 (Bitfield.java:88-93)
    b[33] = c
    b[34:36] = t.to_bytes(2, "big")
    b[36], b[37], b[38], b[39] = r, o, i, k
    return bytes(b).hex()


def H(prefix, n=0):
    """A well-formed 12-char url hash: prefix + base64 digits of n."""
    tail = ""
    for _ in range(12 - len(prefix)):
        tail = ALPHA[n % 64] + tail
        n //= 64
    return prefix + tail


TODAY = 20000
NOW = TODAY * DAY + 12345

kats = []

# --- SegmentTest.testQuery_MultiWordQuery (SegmentTest.java:170-210) --------
# Text "One Two Three Four Five. This is a test text. One two three for five":
#   "five": posintext 5, hitcount 2, posofphrase 100, posinphrase 5
#   "test": posintext 9, hitcount 1, posofphrase 101, posinphrase 4
#   15 words, 3 phrases, 2 title words.  Asserted on the joined reference:
#   posintext 5, hitcount 2, phrasesintext 3, posofphrase 100, posinphrase 5.
url = "kN0WkdoVHAAA"
kats.append({
    "name": "segmenttest_multiword_join",
    "lists": {"TERMfive____": [row(url, c=2, t=5, r=5, o=100, w=15, p=3)],
              "TERMtest____": [row(url, c=1, t=9, r=4, o=101, w=15, p=3)]},
    "include": ["TERMfive____", "TERMtest____"], "exclude": [], "max_distance": 2147483647,
    "now_ms": NOW,
    "expect_rows": [{"h": url, "t": 5, "c": 2, "p": 3, "o": 100, "r": 5,
                     "i": 4}],  # worddistance |5-9| (AbstractReference.java:40-60)
})

# --- J4: by-test join joins the LARGE row with itself (ReferenceContainer.java:440-441)
large = [row(H("LL", j), c=3, t=40, o=120, r=7, i=(17 if j == 50 else 0)) for j in range(100)]
small = [row(H("LL", 50), c=200, t=7, o=101, r=2, u=9, w=999)]
# stepsEnum = 10*(100+1-1) = 1000 > stepsTest = 12*log2(100)*1 = 84 -> by test.
# Output = J6(join(Vars(large[50]), large[50])): features of large[50]; the
# joined distance |40-40| = 0 falls back to the stored distance 17.
kats.append({
    "name": "j4_bytest_selfjoin",
    "lists": {"TERMsmall___": small, "TERMlarge___": large},
    "include": ["TERMsmall___", "TERMlarge___"], "exclude": [], "max_distance": 2147483647,
    "now_ms": NOW,
    "expect_rows": [{"h": H("LL", 50), "c": 3, "t": 40, "o": 120, "r": 7, "u": 2, "w": 15,
                     "i": 17, "a": 15000, "s": 25000, "g": 0, "k": 0}],
    "expect_trace": [{"by_test": 1}],
})

# --- J5/J6: distance byte truncation and maxDistance filter -----------------
# posintext 10 and 310 -> distance 300 (> maxDistance 299 drops it); stored i = 300 & 0xFF = 44
for md, keep in ((299, False), (300, True)):
    kats.append({
        "name": f"j6_distance_truncation_md{md}",
        "lists": {"TERMaaaa____": [row(H("DD", 1), t=10, o=100), row(H("DD", 2), t=5, o=100)],
                  "TERMbbbb____": [row(H("DD", 1), t=310, o=100), row(H("DD", 3), t=5, o=100)]},
        "include": ["TERMaaaa____", "TERMbbbb____"], "exclude": [], "max_distance": md,
        "now_ms": NOW,
        "expect_rows": ([{"h": H("DD", 1), "t": 10, "i": 44}] if keep else []),
    })

# --- J6: re-encoding clamps future dates to today, recomputes freshUntil -----
# a_out = microDateDays(min(now, a*day)); s = max(0, a_out + (today - a_out)*2)
kats.append({
    "name": "j6_date_clamp",
    "lists": {"TERMaaaa____": [row(H("FF", 1), a=25000, t=3), row(H("FF", 2), a=15000, t=3)],
              "TERMbbbb____": [row(H("FF", 1), a=25000, t=4), row(H("FF", 2), a=15000, t=4)]},
    "include": ["TERMaaaa____", "TERMbbbb____"], "exclude": [], "max_distance": 2147483647,
    "now_ms": NOW,
    "expect_rows": [{"h": H("FF", 1), "a": 20000, "s": 20000, "i": 1},
                    {"h": H("FF", 2), "a": 15000, "s": 25000, "i": 1}],
})

# --- J1/J7: exclusion; a missing exclude term disables exclusion entirely ----
inc = [row(H("EE", j), t=1) for j in range(6)]
exc = [row(H("EE", j), t=1) for j in (1, 4, 9)]
kats.append({
    "name": "j7_exclusion",
    "lists": {"TERMinc_____": inc, "TERMexc_____": exc},
    "include": ["TERMinc_____"], "exclude": ["TERMexc_____"], "max_distance": 2147483647,
    "now_ms": NOW,
    "expect_rows": [{"h": H("EE", j)} for j in (0, 2, 3, 5)],
})
kats.append({
    "name": "j1_missing_exclude_term_disables_exclusion",
    "lists": {"TERMinc_____": inc, "TERMexc_____": exc},
    "include": ["TERMinc_____"], "exclude": ["TERMexc_____", "TERMnone____"],
    "max_distance": 2147483647, "now_ms": NOW,
    "expect_rows": [{"h": H("EE", j)} for j in range(6)],
})
kats.append({
    "name": "j1_missing_include_term_empties_result",
    "lists": {"TERMinc_____": inc},
    "include": ["TERMinc_____", "TERMnone____"], "exclude": [], "max_distance": 2147483647,
    "now_ms": NOW, "expect_rows": [],
})

# --- N3 / S1: order-dependent max-distance fold and a negative distance term
# One-term query (rows returned as-is, ReferenceContainer.java:355-370).
# Fold (WordReferenceVars.java:431-445): e0 only initialises P=10 (its od=99
# is ignored, it is the clone); e1 (p=10, od=50) sets A=60; e2 (p=100, od=20):
# dist=|100-60|=40 >= 20 -> unchanged.  D = 40, min distance = 0.
# Profile: allZero + worddistance 10.  All other features equal except
# posintext (10,10,100); url char 11 'A' -> domLengthNormalized 4 -> 252.
#   wd(e0) = (256 - (99<<8)/40) << 10 = -377 << 10 = -386048
#   wd(e1) = (256 - (50<<8)/40) << 10 =  -64 << 10 =  -65536
#   wd(e2) = (256 - (20<<8)/40) << 10 =  128 << 10 =  131072
#   posintext term (shift 0): 256, 256, 0
#   language "de" vs target "en" -> 0; no flags.
fold = [row(H("NN", 1 * 64)[:11] + "A", t=10, i=99, l="de"),
        row(H("NN", 2 * 64)[:11] + "A", t=10, i=50, l="de"),
        row(H("NN", 3 * 64)[:11] + "A", t=100, i=20, l="de")]
kats.append({
    "name": "n3_distance_fold_negative_term",
    "lists": {"TERMfold____": fold},
    "include": ["TERMfold____"], "exclude": [], "max_distance": 2147483647, "now_ms": NOW,
    "profile": {"all_zero": True, "coeff_worddistance": 10}, "language": "en",
    "expect_norm": {"D": 40},
    "expect_hits": [[H("NN", 3 * 64)[:11] + "A", 252 + 0 + 131072],
                    [H("NN", 2 * 64)[:11] + "A", 252 + 256 - 65536],
                    [H("NN", 1 * 64)[:11] + "A", 252 + 256 - 386048]],
})

# --- N2: the first element is a clone whose virtualAge is clamped to today ---
# a = 25000 (future), 15000, 18000; today = 20000.
# min.va = min(20000, 15000, 18000) = 15000; max.va = max(20000, 15000, 18000) = 20000
# date term (allZero, coeff_date 0): ((va - 15000) << 8) / 5000:
#   e0 (raw 25000): 512, e1: 0, e2: (3000*256)/5000 = 153
clamp = [row(H("CC", 1 * 64)[:11] + "A", a=25000, l="de"), row(H("CC", 2 * 64)[:11] + "A", a=15000, l="de"),
         row(H("CC", 3 * 64)[:11] + "A", a=18000, l="de")]
kats.append({
    "name": "n2_clone_virtualage_clamp",
    "lists": {"TERMclmp____": clamp},
    "include": ["TERMclmp____"], "exclude": [], "max_distance": 2147483647, "now_ms": NOW,
    "profile": {"all_zero": True}, "language": "en",
    "expect_hits": [[H("CC", 1 * 64)[:11] + "A", 252 + 512], [H("CC", 3 * 64)[:11] + "A", 252 + 153],
                    [H("CC", 2 * 64)[:11] + "A", 252 + 0]],
})

# --- S1: domLengthNormalized = x << (8/20) = x; int-sum wrap before the long tf term
# url char 11: 'A' (key 0 -> 4 -> 252), 'D' (key 3 -> 20 -> 236)
# coeff_urlcomps = 23: (256 - 0) << 23 = 2^31 wraps to -2^31 in the int sum.
# Flag 28 (appurl) set on both, coeff_appurl = 31: 255 << 31 (int) = -2^31, added as long.
#   e(urlcomps=1, 'A'): int(252 + -2^31) = -2147483396; + (-2^31) long = -4294967044
#   e(urlcomps=2, 'D'): 236 + 0 = 236; + (-2^31) = -2147483412
wrap = [row(H("WW", 1 * 64)[:11] + "A", n=1, l="de", z=1 << 28), row(H("WW", 2 * 64)[:11] + "D", n=2, l="de", z=1 << 28)]
kats.append({
    "name": "s1_domlength_and_int_long_boundary",
    "lists": {"TERMwrap____": wrap},
    "include": ["TERMwrap____"], "exclude": [], "max_distance": 2147483647, "now_ms": NOW,
    "profile": {"all_zero": True, "coeff_urlcomps": 23, "coeff_appurl": 31}, "language": "en",
    "expect_hits": [[H("WW", 2 * 64)[:11] + "D", 236 - 2147483648],
                    [H("WW", 1 * 64)[:11] + "A", -2147483396 - 2147483648]],
})

# --- T1: top-k order (score desc, ByteArray.hashCode desc); equal (score, hash)
# is rejected by the TreeSet, so the later (larger url hash) posting vanishes.
# "Aa" and "BB" have equal Java hash codes (65*31+97 == 66*31+66).
def java_hash(s):  # ByteArray.hashCode (ByteArray.java:80-84), Java int
    h = 0
    for ch in s.encode():
        h = (31 * h + ch) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


# container order (ascending url hash): tieAAAa.. < tieAAAc.. < tieAABB..
tie = [row("tieAAAaAAAAA", l="de"), row("tieAAAcAAAAA", l="de"), row("tieAABBAAAAA", l="de")]
assert java_hash("tieAAAaAAAAA") == java_hash("tieAABBAAAAA")
ha, hc = java_hash("tieAAAaAAAAA"), java_hash("tieAAAcAAAAA")
order = ["tieAAAcAAAAA", "tieAAAaAAAAA"] if hc > ha else ["tieAAAaAAAAA", "tieAAAcAAAAA"]
kats.append({
    "name": "t1_tiebreak_and_treeset_dedupe",
    "lists": {"TERMtie_____": tie},
    "include": ["TERMtie_____"], "exclude": [], "max_distance": 2147483647, "now_ms": NOW,
    "profile": {"all_zero": True}, "language": "en",
    # all scores 252; higher hashCode first; tieAABBAAAAA ties tieAAAaAAAAA on
    # (score, hash) and arrives later, so the TreeSet rejects it.
    "expect_hits": [[order[0], 252], [order[1], 252]],
})

# --- WordReferenceVarsTest.testMin (WordReferenceVarsTest.java:40-95) ---------
kats.append({
    "name": "wordreferencevarstest_min",
    "vars_test": True,
    "expect": {"min_posintext": 5, "min_distance": 5, "max_posintext": 30, "max_distance": 25,
               "reverse_posintext": 30, "reverse_distance": 25},
})

# --- ReferenceContainerTest.testAdd (ReferenceContainerTest.java:51-100) -------
kats.append({
    "name": "referencecontainertest_add_distance_roundtrip",
    "container_add_test": True,
    "expect": {"distance": 9},
})

out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
with open(out, "w") as f:
    json.dump({"today": TODAY, "now_ms": NOW, "kats": kats}, f, indent=1)
print("wrote", out, len(kats), "kats")
