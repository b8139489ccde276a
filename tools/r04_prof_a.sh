# Round-4 profiles, part 1: C2 and C5 custom at commit 9bb1395.
PROF_HEAD=9bb1395 bash tools/prof_r04.sh r04 "C2 C5"
