# Round-4 profiles, part 2: C3 and C4 at commit 88b79af.
PROF_HEAD=88b79af bash tools/prof_r04.sh r04 "C3 C4"
