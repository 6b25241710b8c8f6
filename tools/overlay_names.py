"""Build-container tool: which names do the NON-replaced reference modules take from the replaced ones?

The drop-in (humanoid-real-time-retarget_amd/) replaces a set of reference modules (same dotted paths).  Every
other reference module and entry point -- retarget/utils/*, the sim_*_teleop scripts, mocap_control_arm.py,
vedo_visualizer/*, the asset generators, zero_pose_transform.py, rotation_test.py -- keeps running unchanged and
takes names from the replaced modules in three ways, all resolved here statically (ast, nothing is imported or run):

* ``from X import a, b``            -> X must export a and b (or have submodules a, b);
* ``from X import *`` then ``a``     -> every free name the module uses that the REFERENCE X star-exports (its
                                        ``__all__`` or, without one, every public top-level binding, imports
                                        included, star re-exports followed) must be star-exported by the drop-in X.
                                        When several star imports provide a name, the last one in the file wins;
* ``Cls.attr`` on a class imported from X (``SkeletonState.zero_pose``, ``RobotZeroPose.from_urdf``) -> the
                                        drop-in class must have attr.

Writes tests/golden/overlay_names.json; tests/test_host_logic.py::test_overlay_exports_every_name_the_reference_uses
asserts the drop-ins export every entry.  Usage: python tools/overlay_names.py [/root/reference]
"""
from __future__ import annotations

import ast
import builtins
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROP = os.path.join(REPO, "humanoid-real-time-retarget_amd")
OUT = os.path.join(REPO, "tests", "golden", "overlay_names.json")
MIRRORED_TOPS = ("poselib", "retarget", "robot_kinematics_model")


def modules(root, tops=None):
    out = {}
    for d, _, files in os.walk(root):
        for f in files:
            if not f.endswith(".py"):
                continue
            rel = os.path.relpath(os.path.join(d, f), root)
            parts = rel[:-3].split(os.sep)
            if parts[-1] == "__init__":
                parts = parts[:-1]
            if not parts or (tops and parts[0] not in tops):
                continue
            out[".".join(parts)] = os.path.join(d, f)
    return out


def resolve(mod, is_pkg, node):
    """Absolute dotted name of an ImportFrom's module."""
    if not node.level:
        return node.module
    base = mod.split(".") if is_pkg else mod.split(".")[:-1]
    base = base[:len(base) - (node.level - 1)] if node.level > 1 else base
    return ".".join(base + ([node.module] if node.module else []))


def is_main_guard(stmt):
    return (isinstance(stmt, ast.If) and isinstance(stmt.test, ast.Compare)
            and isinstance(stmt.test.left, ast.Name) and stmt.test.left.id == "__name__")


class Ref:
    def __init__(self, root):
        self.root = root
        self.mods = modules(root)
        self.trees = {}
        self._star = {}

    def tree(self, m):
        if m not in self.trees:
            self.trees[m] = ast.parse(open(self.mods[m], encoding="utf-8").read(), self.mods[m])
        return self.trees[m]

    def is_pkg(self, m):
        return self.mods[m].endswith("__init__.py")

    def star_exports(self, m, stack=()):
        """Names ``from m import *`` binds (module-level statements outside the __main__ guard)."""
        if m in self._star:
            return self._star[m]
        if m not in self.mods or m in stack:
            return set()
        t = self.tree(m)
        names, explicit = set(), None
        for stmt in self._toplevel(t.body):
            if isinstance(stmt, ast.Assign) and any(isinstance(x, ast.Name) and x.id == "__all__" for x in stmt.targets):
                try:
                    explicit = set(ast.literal_eval(stmt.value))
                except ValueError:
                    pass
            for n in self._binds(stmt):
                names.add(n)
            if isinstance(stmt, ast.ImportFrom) and any(a.name == "*" for a in stmt.names):
                names |= self.star_exports(resolve(m, self.is_pkg(m), stmt), stack + (m,))
        out = explicit if explicit is not None else {n for n in names if not n.startswith("_")}
        self._star[m] = out
        return out

    def _toplevel(self, body):
        for stmt in body:
            if is_main_guard(stmt):
                continue
            if isinstance(stmt, (ast.If, ast.Try)):
                for sub in (getattr(stmt, "body", []), getattr(stmt, "orelse", []),
                            getattr(stmt, "finalbody", []), *[h.body for h in getattr(stmt, "handlers", [])]):
                    yield from self._toplevel(sub)
            else:
                yield stmt

    @staticmethod
    def _binds(stmt):
        if isinstance(stmt, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            return [stmt.name]
        if isinstance(stmt, ast.Import):
            return [a.asname or a.name.split(".")[0] for a in stmt.names]
        if isinstance(stmt, ast.ImportFrom):
            return [a.asname or a.name for a in stmt.names if a.name != "*"]
        out = []
        targets = stmt.targets if isinstance(stmt, ast.Assign) else \
            [stmt.target] if isinstance(stmt, (ast.AnnAssign, ast.AugAssign)) else []
        for t in targets:
            for n in ast.walk(t):
                if isinstance(n, ast.Name):
                    out.append(n.id)
        return out


def local_bindings(tree):
    """Every name a module binds anywhere (params, assignments, defs, imports, loop/with/except targets)."""
    out = set()
    for n in ast.walk(tree):
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, ast.arg):
            out.add(n.arg)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
        elif isinstance(n, ast.Import):
            out.update(a.asname or a.name.split(".")[0] for a in n.names)
        elif isinstance(n, ast.ImportFrom):
            out.update(a.asname or a.name for a in n.names if a.name != "*")
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
    return out


# names the scan finds that the drop-in deliberately leaves out, with the reason (SURVEY.md §2 scope)
OUT_OF_SCOPE = {
    "SkeletonTree.from_mjcf": "offline MJCF import (SURVEY §2 row 3); only poselib's own broken test_skeleton.py uses it",
}


def provides(ref, mod, name):
    """Does the REFERENCE module itself bind ``name`` (a top-level name, star export, or submodule)?"""
    if mod not in ref.mods:
        return False
    if name in ref.star_exports(mod) or f"{mod}.{name}" in ref.mods:
        return True
    return any(name in Ref._binds(st) for st in ref._toplevel(ref.tree(mod).body))


def class_has(ref, mod, dotted):
    """Does the reference class (defined in ``mod`` or imported there) have the attribute, through its bases?"""
    cls, attr = dotted.split(".", 1)
    seen = set()

    def find(m, c):
        if (m, c) in seen or m not in ref.mods:
            return None
        seen.add((m, c))
        for node in ast.walk(ref.tree(m)):
            if isinstance(node, ast.ClassDef) and node.name == c:
                return m, node
        for node in ast.walk(ref.tree(m)):     # re-exported: follow the import
            if isinstance(node, ast.ImportFrom):
                src = resolve(m, ref.is_pkg(m), node)
                for a in node.names:
                    if a.name == "*" or (a.asname or a.name) == c:
                        hit = find(src, c if a.name == "*" else a.name)
                        if hit:
                            return hit
        return None

    def has(m, c):
        hit = find(m, c)
        if not hit:
            return False
        m2, node = hit
        for st in node.body:
            if isinstance(st, (ast.FunctionDef, ast.AsyncFunctionDef)) and st.name == attr:
                return True
            if attr in Ref._binds(st):
                return True
        return any(has(m2, b.id) for b in node.bases if isinstance(b, ast.Name))
    return has(mod, cls)


def scan(ref_root):
    ref = Ref(ref_root)
    drop = modules(DROP, MIRRORED_TOPS)
    replaced = sorted(m for m in ref.mods if m in drop)
    req = {}          # (module, name) -> set of "file:line"
    submods = {}      # module names imported from replaced packages that the drop-in does not ship
    class_attrs = {}  # (module, "Cls.attr") -> users
    builtin_names = set(dir(builtins))

    def need(table, key, where):
        table.setdefault(key, set()).add(where)

    for m in sorted(ref.mods):
        if m in drop:
            continue
        t = ref.tree(m)
        rel = os.path.relpath(ref.mods[m], ref_root)
        used = {}
        for n in ast.walk(t):
            if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
                used.setdefault(n.id, n.lineno)
        free = {k: v for k, v in used.items() if k not in local_bindings(t) and k not in builtin_names}
        providers = {}   # free name -> replaced module whose star import binds it last
        imported_cls = {}
        stars = sorted((n for n in ast.walk(t) if isinstance(n, ast.ImportFrom)), key=lambda n: n.lineno)
        for node in stars:
            src = resolve(m, ref.is_pkg(m), node)
            if src not in ref.mods and src not in drop:
                continue
            for a in node.names:
                if a.name == "*":
                    for name in ref.star_exports(src):
                        if name in free:
                            providers[name] = (src, node.lineno)
                    continue
                if src not in drop:
                    continue
                sub = f"{src}.{a.name}"
                if sub in ref.mods:                      # a submodule, not an attribute
                    if sub not in drop:
                        need(submods, sub, f"{rel}:{node.lineno}")
                    continue
                need(req, (src, a.name), f"{rel}:{node.lineno}")
                imported_cls[a.asname or a.name] = src
            for a in node.names:   # names bound by this explicit import shadow earlier star providers
                if a.name != "*":
                    providers.pop(a.asname or a.name, None)
        for name, (src, line) in providers.items():
            if src in drop:
                need(req, (src, name), f"{rel}:{free[name]} (via `from {src} import *` at :{line})")
                if name[:1].isupper():
                    imported_cls[name] = src
        for n in ast.walk(t):
            if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name) and n.value.id in imported_cls \
                    and n.value.id[:1].isupper():
                need(class_attrs, (imported_cls[n.value.id], f"{n.value.id}.{n.attr}"), f"{rel}:{n.lineno}")
    star_sources = sorted({src for (src, _name) in req if any("import *" in u for u in req[(src, _name)])})
    broken = {k: v for k, v in req.items() if not provides(ref, k[0], k[1])}
    names = {k: v for k, v in req.items() if k not in broken}
    attrs_ok = {k: v for k, v in class_attrs.items() if class_has(ref, k[0], k[1])}
    return {
        "about": "names that non-replaced reference modules take from replaced ones (tools/overlay_names.py)",
        "replaced_modules": replaced,
        "names": [{"module": k[0], "name": k[1], "used_by": sorted(v)} for k, v in sorted(names.items())],
        "class_attributes": [{"module": k[0], "attr": k[1], "used_by": sorted(v),
                              **({"out_of_scope": OUT_OF_SCOPE[k[1]]} if k[1] in OUT_OF_SCOPE else {})}
                             for k, v in sorted(attrs_ok.items())],
        # a replaced module that some caller star-imports must star-export everything the reference's does
        "star_exports": {m: sorted(ref.star_exports(m)) for m in star_sources},
        "reference_submodules_not_replaced": [{"module": k, "used_by": sorted(v)} for k, v in sorted(submods.items())],
        "broken_in_reference": [{"module": k[0], "name": k[1], "used_by": sorted(v)} for k, v in sorted(broken.items())]
        + [{"module": k[0], "attr": k[1], "used_by": sorted(v)} for k, v in sorted(class_attrs.items())
           if k not in attrs_ok],
    }


def main():
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    res = scan(ref_root)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, sort_keys=False)
        f.write("\n")
    print(f"{len(res['names'])} names, {len(res['class_attributes'])} class attributes, "
          f"{len(res['reference_submodules_not_replaced'])} unreplaced submodules -> {OUT}")


if __name__ == "__main__":
    main()
