# Round 4: per-entity-class dof spread inside the 4x4x4 bricks of the reference numbering (C4 drop-in):
# could a lattice map be stored as 4 class bases + 16-bit offsets?  python3 profiles/r4_mapspread.py <n>
import sys, numpy as np
sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo')
import helpers
E = helpers.load_pkg()
n = int(sys.argv[1])
m = E.Mesh.MakeCartesian3D(n, n, n, sfc_ordering=True)
fes = E.H1Space(m, 2, E.NUMBERING_ENTITY)
gm = fes.gather_map()
gm = np.where(gm < 0, -1 - gm, gm)
perm = fes.element_order_faces()
nv = (n + 1) ** 3
ne_edges = 3 * n * (n + 1) ** 2
nf = 3 * n * n * (n + 1)
# entity numbering at p = 2: [vertices | edges (1 dof each) | faces (1 each) | interiors (1 each)]
bounds = np.array([0, nv, nv + ne_edges, nv + ne_edges + nf, fes.ndofs])
nb = len(perm) // 64
g = gm[perm[: nb * 64]].reshape(nb, 64 * 27)
spread = []
for c in range(4):
    lo, hi = bounds[c], bounds[c + 1]
    mask = (g >= lo) & (g < hi)
    big = np.where(mask, g, np.iinfo(np.int32).min).max(axis=1)
    small = np.where(mask, g, np.iinfo(np.int32).max).min(axis=1)
    sp = big - small
    spread.append((int(np.median(sp)), int(sp.max())))
    fits = sp < 65536 if c == 0 else fits & (sp < 65536)
print("bricks whose four classes fit 16-bit offsets:", round(float(fits.mean()), 4))
print(n, "blocks", nb, "ndofs", fes.ndofs, "per-class spread (median, max):", dict(zip(["vertex", "edge", "face", "interior"], spread)))
