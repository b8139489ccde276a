# Round-4 profiles, part 1: C2 and C5 custom at commit 88b79af.
PROF_HEAD=88b79af bash tools/prof_r04.sh r04 "C2 C5"
