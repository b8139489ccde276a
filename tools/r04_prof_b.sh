# Round-4 profiles, part 2: C3 and C4 at commit f9c622f.
PROF_HEAD=f9c622f bash tools/prof_r04.sh r04 "C3 C4"
