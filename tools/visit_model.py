"""Model of the sphere kernel's march visits: for random 32x8 tiles of the 4K
64-sphere frame, simulate the march in numpy float32 (approximate pass threshold; counts only)
and count per step the spheres the kernel visits (cull cone + march window with the half-width
sqrt(rr^2 - dmin^2), low end every 2nd step, SGPR-slot waves visit all their culled spheres)
against those that pass for some lane.
    python tools/visit_model.py [rotation hrotation] [--round1-window]
"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sfml-software-raytracer_amd'))
import scenes
f32 = np.float32
W, H = 3840, 2160
args = [a for a in sys.argv[1:] if not a.startswith('--')]
ROUND1 = '--round1-window' in sys.argv
pose = tuple(float(x) for x in args[:2]) if len(args) > 1 else (0.0, 0.0)
sc = scenes.lcg64().posed(*pose)
S = sc.spheres.astype(f32); n = len(S)
cam = np.array(sc.cam_pos, f32)
def rx(v, a):
    s, c = np.sin(f32(a)), np.cos(f32(a)); x, y, z = v
    return np.array([x, y*c - z*s, y*s + z*c], f32)
def ry(v, a):
    s, c = np.sin(f32(a)), np.cos(f32(a)); x, y, z = v
    return np.array([x*c + z*s, y, -x*s + z*c], f32)
up = ry(rx(np.array([0,-1,0],f32), -sc.hrotation), sc.rotation)
fw = ry(rx(np.array([0,0,1],f32), -sc.hrotation), sc.rotation)
rt = ry(np.array([1,0,0],f32), sc.rotation)
fovh, fovv = f32(sc.fov_h), f32(sc.fov_v)
hs, hi_ = -fovh, fovh / f32(W) * f32(2); vs, vi = -fovv, fovv / f32(H) * f32(2)
def dirs(ii, jj):
    h = hs + hi_ * ii.astype(f32); v = vs + jj.astype(f32) * vi
    d = (fw[None] + rt[None] * h[:, None]) + up[None] * v[:, None]
    l = np.sqrt((d[:,0]*d[:,0] + d[:,1]*d[:,1]) + d[:,2]*d[:,2])
    return d / l[:, None]
cs, rs = S[:, :3], S[:, 3]
spass = (rs - f32(0.01))**2  # approx threshold
reach = max(np.linalg.norm(cam), (np.linalg.norm(cs, axis=1) + rs).max())
margin = f32(1e-3 * reach + 1e-4)
rng = np.random.default_rng(0)
TX, TY = 32, 8
SLOTS = 2
ntiles = 3000
tot_steps = tot_win = tot_min = tot_slot = 0; tot_win_onlymin=0
for t in range(ntiles):
    tx = rng.integers(W // TX); ty = rng.integers(H // TY)
    jj, ii = np.meshgrid(np.arange(ty*TY, ty*TY+TY), np.arange(tx*TX, tx*TX+TX), indexing='ij')
    ii = ii.ravel(); jj = jj.ravel()
    d = dirs(ii, jj)
    # first iteration from cam
    dc = np.linalg.norm(cam[None] - cs, axis=1)
    ok = rs - dc > 0.01
    l0 = (rs - dc)[ok].max() if ok.any() else f32(0)
    p = cam[None] + d * f32(l0)
    mv = np.full(len(ii), l0 > 0); tacc = np.full(len(ii), f32(l0))
    # cone
    ic = tx*TX + (TX/2 - .5); jc = ty*TY + 3.5
    a = dirs(np.array([ic]), np.array([jc]))[0].astype(np.float64)
    dd = d.astype(np.float64)
    sin_t = min(1.0, np.linalg.norm(np.cross(dd, a), axis=1).max() + 1e-5); cos_t = np.sqrt(1 - sin_t**2)
    w = (cs - cam[None]).astype(np.float64); wl = np.linalg.norm(w, axis=1)
    rr = rs + margin + 4e-6 * wl
    tt = w @ a; perp = np.linalg.norm(w - tt[:, None] * a[None], axis=1)
    side = tt * cos_t + perp * sin_t >= -rr
    sa = perp * cos_t - tt * sin_t; sb = perp * cos_t + tt * sin_t
    inc = (wl <= rr) | (side & (sa <= rr))
    upb = np.where(sa >= 0, tt*cos_t + perp*sin_t, wl); dn = np.where(sb >= 0, tt*cos_t - perp*sin_t, -wl)
    if ROUND1:
        h = rr
    else:
        dmin = np.maximum(0.0, np.minimum(sa, sb) - 4e-6 * wl)
        h = np.sqrt(np.maximum(0.0, (rr - dmin) * (rr + dmin))) * 1.00001
    lo = dn - (h + margin); hi = upb + (h + margin)
    m = inc.copy()
    slots = m.sum() <= SLOTS
    trips = 1; tlo = 0.0
    while mv.any():
        if trips % 2 == 1: tlo = tacc[mv].min()
        thi = tacc.max()
        win = m & (lo < thi) & (hi > tlo)
        e = p[:, None, :] - cs[None]
        ss = (e[...,0]*e[...,0] + e[...,1]*e[...,1]) + e[...,2]*e[...,2]
        passm = (ss < spass[None]) & mv[:, None]
        need = passm.any(axis=0)
        assert not (need & ~m).any()
        tot_steps += 1; tot_min += need.sum(); tot_win += (m.sum() if slots else win.sum())
        # step
        L = np.where(passm, rs[None] - np.sqrt(ss), f32(0)).max(axis=1).astype(f32)
        p = np.where(mv[:, None], p + d * L[:, None], p)
        tacc = np.where(mv, tacc + L, tacc); mv = mv & (L > 0)
        trips += 1
print(pose, 'steps/tile', tot_steps/ntiles, 'visits/step', tot_win/tot_steps, 'needed/step', tot_min/tot_steps)
