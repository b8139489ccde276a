# Round-4 profiles, part 1: C2 and C5 custom at commit 8287044.
PROF_HEAD=8287044 bash tools/prof_r04.sh r04 "C2 C5"
