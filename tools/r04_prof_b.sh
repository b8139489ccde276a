# Round-4 profiles, part 2: C3 and C4 at commit 9bb1395.
PROF_HEAD=9bb1395 bash tools/prof_r04.sh r04 "C3 C4"
