import sys, numpy as np
sys.path.insert(0, "/root/repo")
from oracle import np_select as S
hits = {"mom5": 0}
orig = S._median_of_median5
def mm(v, o, num):
    hits["mom5"] += 1
    return orig(v, o, num)
S._median_of_median5 = mm
def killer(n):
    # median-of-3 killer permutation (Musser)
    k = n // 2
    a = np.zeros(n)
    for i in range(1, k + 1):
        if i % 2 == 1:
            a[i - 1] = i; a[i] = k + i
        a[k + i - 1] = 2 * i
    return a
rng = np.random.default_rng(0)
bad = 0; tot = 0
for trial in range(2500):
    n = int(rng.choice([1,2,3,4,5,6,7,8,10,16,33,64,100,257,1000,5000]))
    kind = trial % 6
    if kind == 0:
        x = rng.choice([-0.0, 0.0], n)
    elif kind == 1:
        x = rng.choice([-1.0, -0.0, 0.0, 1.0, 2.0], n)
    elif kind == 2:
        x = rng.standard_normal(n); m = rng.random(n) < 0.3; x[m] = rng.choice([-0.0, 0.0], m.sum())
    elif kind == 3:
        x = np.sort(rng.choice([-1.0, -0.0, 0.0, 1.0], n))
        if trial % 12 == 3: x = x[::-1].copy()
    elif kind == 4:
        x = killer(n) - n // 2; x[x == 0] = -0.0; x[rng.random(n) < 0.2] = 0.0
    else:
        x = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]).astype(float) - n // 4
        x[x == 0] = rng.choice([-0.0, 0.0], (x == 0).sum())
    for q in (1, 99, 50, 25, 0, 100, 5):
        vi = (n - 1) * (q / 100)
        if vi >= n - 1:
            kth = np.unique([0, -1, -1, -1])
        else:
            i = int(np.floor(vi)); kth = np.unique([0, -1, i, i + 1])
        a = x.copy(); a.partition(kth)
        b = S.partition(x, kth)
        tot += 1
        if not np.array_equal(a.view(np.uint64), b.view(np.uint64)):
            bad += 1
            if bad < 5: print("mismatch", n, q, kind)
        pa = np.argpartition(x, kth)
        ab = np.array(S.partition(x.copy(), kth))
print("total", tot, "bad", bad, hits)
