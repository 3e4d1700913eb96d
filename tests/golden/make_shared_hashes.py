"""Writes tests/golden/shared_hashes.json: an SDFEditor save (serde layout of
sdf_editor.rs:131-167) whose Floats share hashes the way the reference's
editor produces them -- `#[derive(Clone)]` on Shape/Float copies the hash
(primitives.rs:203-211), and a hand-edited save can repeat any hash.

* union "objects": c2's sphere and box, then a clone of the box (every hash
  shared) with a different position value in the file (compile keeps the
  first value; a refresh writes the last one, primitives.rs:117-129,153-156);
* the sphere's surface colour shares its hash with the box's spec colour;
* the box's rotation x and z share one hash (one slot inside one V3);
* union "light" (c2's light and floor) is left alone.

Run: python tests/golden/make_shared_hashes.py
"""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from compute_path_tracer_amd import scenes  # noqa: E402


def main() -> None:
    ed = scenes.c2_sphere_box_torus()
    d = json.loads(ed.dumps())
    a, b, light = d["header_unions"]
    sphere = a["children_shapes"][1]
    box = copy.deepcopy(b["children_shapes"][1])
    obj = {"name": "objects", "transform": a["transform"], "union_type": "Union", "children_unions": [],
           "children_shapes": [sphere, box]}
    box["material"]["specular_color"] = copy.deepcopy(sphere["material"]["color"])
    box["material"]["specular_color"]["name"] = "Spec color"
    box["transform"]["rotation"]["z"]["hash"] = box["transform"]["rotation"]["x"]["hash"]
    clone = copy.deepcopy(box)
    clone["name"] = "box clone"
    clone["transform"]["position"]["x"]["val"] = -1.6  # same hash: the compile keeps 0.8
    obj["children_shapes"].append(clone)
    d["header_unions"] = [obj, light]
    d["save_name"] = "shared_hashes"
    with open(os.path.join(os.path.dirname(__file__), "shared_hashes.json"), "w") as f:
        json.dump(d, f, indent=1)


if __name__ == "__main__":
    main()
