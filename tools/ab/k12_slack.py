# A/B patch: the Gram waves wait for one more published step than needed (a pair is read only once its K1 wave
# has finished the NEXT step too): if a read-before-write race is the cause of NaN Grams, this hides it.
p = "sysid_kernels.h"
s = open(p).read()
old = "const int v = (int)(p & (K1_WAVES - 1)), need = (int)(p / K1_WAVES) + 1;"
assert old in s
s = s.replace(old, "const int v = (int)(p & (K1_WAVES - 1)), need = min((int)(p / K1_WAVES) + 2, (int)((np + K1_WAVES - 1 - v) / K1_WAVES));")
open(p, "w").write(s)
