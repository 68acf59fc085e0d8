"""Mutation fuzz of pt_scene_load_json (CPU): random JSON edits of a bundled scene, each loaded in a
child process so a crash shows as its exit status.  usage: scene_loader_fuzz.py seed count [scene.json]
(run from a scratch directory holding copies of tests/scenes/Models and Textures)."""
import json, random, subprocess, sys, copy, os
base = json.load(open(sys.argv[3] if len(sys.argv) > 3 else '/root/repo/tests/scenes/cornell.json'))
random.seed(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
vals = [0, -1, 1e38, -1e38, float('nan'), float('inf'), "x", None, [], {}, [1], [1, 2], [1, 2, 3, 4], 2**31, -2**31, 1e-45, True, "", [float('nan')]*3]
def mutate(d, depth=0):
    d = copy.deepcopy(d)
    for _ in range(random.randint(1, 3)):
        path = []
        cur = d
        while isinstance(cur, (dict, list)) and cur and random.random() < 0.8:
            k = random.choice(list(cur.keys())) if isinstance(cur, dict) else random.randrange(len(cur))
            path.append((cur, k)); cur = cur[k]
        if not path: continue
        parent, k = path[-1]
        r = random.random()
        if r < 0.6: parent[k] = random.choice(vals)
        elif r < 0.8 and isinstance(parent, dict): del parent[k]
        else: parent[k] = copy.deepcopy(parent[k]) if not isinstance(parent[k], list) else parent[k] * 2
    return d
crashes = 0
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 100):
    m = mutate(base)
    p = f'/tmp/fuzz/s_{i}.json'
    s = json.dumps(m).replace('NaN', 'NaN').replace('Infinity', '1e999')
    open(p, 'w').write(s)
    r = subprocess.run([sys.executable, '-c', f"""
import sys; sys.path.insert(0, '/root/repo')
import os; os.environ['PT_AMD_NO_TORCH']='1'
from cuda_pathtracer_amd import _native as N
import ctypes as C
h = C.c_void_p()
rc = N.lib().pt_scene_load_json(b'{p}', C.byref(h))
if rc == 0: N.lib().pt_scene_free(h)
print(rc)
"""], capture_output=True, text=True, timeout=60)
    if r.returncode != 0:
        crashes += 1
        print('CRASH', i, r.returncode, s[:300].replace(chr(10),' '), r.stderr[-300:])
print('crashes', crashes)
