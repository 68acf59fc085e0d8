"""Scene variants of cornell.json for cost attribution (dev tool): writes JSON files to argv[1]."""
import json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
base = json.loads((ROOT / "tests" / "scenes" / "cornell.json").read_text())
out = Path(sys.argv[1]); out.mkdir(parents=True, exist_ok=True)
def w(name, sc): (out / f"{name}.json").write_text(json.dumps(sc))
w("base", base)
s = json.loads(json.dumps(base)); s["Objects"] = [o for o in s["Objects"] if o["TYPE"] != "sphere"]; w("nosphere", s)
s = json.loads(json.dumps(base)); s["Materials"]["specular_white"] = {"TYPE": "Diffuse", "RGB": [0.98, 0.98, 0.98]}; w("diffsphere", s)
s = json.loads(json.dumps(base)); s["Objects"] = [o for o in s["Objects"] if o["MATERIAL"] != "diffuse_white" or o["TRANS"] != [0.0, 10.0, 0.0]]; w("noceiling", s)
