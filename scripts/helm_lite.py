#!/usr/bin/env python3
"""Render this repo's Helm charts without a helm binary (CPU tests, no network).

A small interpreter for the Go-template + Sprig subset the charts under core/helm-charts use:
``if / else if / else / end``, ``with``, ``range``, ``define`` / ``include``, variables
(``$x := ...``, ``$``), pipelines and parenthesised sub-expressions, and the functions
and, or, not, eq, ne, default, quote, printf, print, include, nindent, indent, toYaml,
fromYaml, splitList, last, trunc, trimSuffix, contains, int, index, sha256sum, list,
deepCopy, set, add1.
Anything else raises, so a template that outgrows the subset fails its test loudly instead
of rendering wrong.  Values are merged like ``helm --values a --values b --set k=v``.

  python scripts/helm_lite.py core/helm-charts/vllm -f core/helm-charts/vllm/mi355x-values.yaml \\
      --set platform=openshift --set ingress.enabled=true
"""

from __future__ import annotations

import copy
import hashlib
import json
import os
import re
import sys
from typing import Any, Dict, List, Optional

import yaml

# ----------------------------------------------------------------------------- lexing

_ACTION = re.compile(r"\{\{(-?)(.*?)(-?)\}\}", re.S)


def _lex(src: str):
    """[("text", s) | ("act", body)] with Go's {{- / -}} whitespace trimming applied."""
    out = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1) == "-":
            text = text.rstrip(" \t\r\n")
        out.append(["text", text])
        out.append(["act", m.group(2).strip(), m.group(3) == "-"])
        pos = m.end()
    out.append(["text", src[pos:]])
    res = []
    trim_next = False
    for item in out:
        if item[0] == "text":
            t = item[1].lstrip(" \t\r\n") if trim_next else item[1]
            trim_next = False
            res.append(("text", t))
        else:
            trim_next = item[2]
            body = item[1]
            if body.startswith("/*"):
                continue
            res.append(("act", body))
    return res


_TOK = re.compile(r'''\s*(?:
    (?P<str>"(?:[^"\\]|\\.)*"|`[^`]*`)
  | (?P<num>-?\d+(?:\.\d+)?)
  | (?P<decl>:=|=)
  | (?P<punct>[()|,])
  | (?P<word>[$.]?[A-Za-z_0-9$.]*[A-Za-z_0-9]|\$|\.)
)''', re.X)


def _tokens(s: str) -> List[str]:
    out, pos = [], 0
    s = s.strip()
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            raise ValueError(f"cannot tokenize {s[pos:]!r} in {s!r}")
        out.append(m.group(m.lastgroup))
        pos = m.end()
    return out


# ----------------------------------------------------------------------------- parsing

class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Act(Node):
    def __init__(self, expr):
        self.expr = expr


class Block(Node):
    def __init__(self, kind, expr):
        self.kind, self.expr = kind, expr
        self.body: List[Node] = []
        self.elifs: List = []          # [(expr, body)]
        self.other: Optional[List[Node]] = None


def _parse(items, defines: Dict[str, List[Node]]) -> List[Node]:
    root: List[Node] = []
    stack: List = [(None, root)]

    def cur() -> List[Node]:
        return stack[-1][1]

    for kind, val in items:
        if kind == "text":
            if val:
                cur().append(Text(val))
            continue
        head = val.split(None, 1)
        word = head[0] if head else ""
        rest = head[1] if len(head) > 1 else ""
        if word in ("if", "with", "range"):
            b = Block(word, rest)
            cur().append(b)
            stack.append((b, b.body))
        elif word == "define":
            name = json.loads(rest.strip())
            b = Block("define", name)
            stack.append((b, b.body))
        elif word == "else":
            b = stack[-1][0]
            stack.pop()
            if rest.startswith("if "):
                body: List[Node] = []
                b.elifs.append((rest[3:], body))
                stack.append((b, body))
            else:
                b.other = []
                stack.append((b, b.other))
        elif word == "end":
            b, _ = stack.pop()
            if b.kind == "define":
                defines[b.expr] = b.body
        else:
            cur().append(Act(val))
    if len(stack) != 1:
        raise ValueError("unbalanced template blocks")
    return root


# ----------------------------------------------------------------------------- evaluation

def _truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return bool(v)


def _str(v) -> str:
    if v is None:
        return ""
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    return str(v)


def _printf(fmt, *args):
    conv = re.sub(r"%v", "%s", fmt)
    return conv % tuple(_str(a) if isinstance(a, (dict, list, bool, type(None))) else a
                        for a in args)


def _to_yaml(v):
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=False).rstrip("\n")


class Renderer:
    def __init__(self, chart_dir: str, values: dict, release: str = "rel",
                 namespace: str = "default"):
        self.defines: Dict[str, List[Node]] = {}
        self.templates: Dict[str, List[Node]] = {}
        with open(os.path.join(chart_dir, "Chart.yaml")) as f:
            chart = yaml.safe_load(f)
        tdir = os.path.join(chart_dir, "templates")
        for name in sorted(os.listdir(tdir)):
            path = os.path.join(tdir, name)
            if not os.path.isfile(path):
                continue
            with open(path) as f:
                nodes = _parse(_lex(f.read()), self.defines)
            if name.endswith((".yaml", ".yml")):
                self.templates[name] = nodes
        self.root = {"Values": values, "Chart": {"Name": chart.get("name"),
                                                 "Version": chart.get("version"),
                                                 "AppVersion": chart.get("appVersion")},
                     "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
                     "Template": {"BasePath": "templates"}}
        self.funcs = {
            "and": self._and, "or": self._or, "not": lambda v: not _truthy(v),
            "eq": lambda a, *b: any(a == x for x in b), "ne": lambda a, b: a != b,
            "default": lambda d, v=None: v if _truthy(v) else d,
            "quote": lambda *v: " ".join(json.dumps(_str(x)) for x in v),
            "printf": _printf, "print": lambda *v: "".join(_str(x) for x in v),
            "nindent": lambda n, s: "\n" + self._indent(n, s),
            "indent": lambda n, s: self._indent(n, s),
            "toYaml": _to_yaml, "fromYaml": lambda s: yaml.safe_load(s) or {},
            "splitList": lambda sep, s: _str(s).split(sep),
            "last": lambda l: l[-1] if l else None,
            "trunc": lambda n, s: _str(s)[:n], "trimSuffix": lambda suf, s: _str(s)[:-len(suf)]
            if suf and _str(s).endswith(suf) else _str(s),
            "contains": lambda sub, s: _str(sub) in _str(s), "int": lambda v: int(v or 0),
            "index": self._index, "sha256sum": lambda s: hashlib.sha256(_str(s).encode()).hexdigest(),
            "list": lambda *v: list(v), "include": self._include,
            "deepCopy": copy.deepcopy, "set": _sprig_set, "add1": lambda v: int(v or 0) + 1,
        }

    # -- functions
    @staticmethod
    def _and(*a):
        for x in a:
            if not _truthy(x):
                return x
        return a[-1]

    @staticmethod
    def _or(*a):
        for x in a:
            if _truthy(x):
                return x
        return a[-1]

    @staticmethod
    def _indent(n, s):
        return "\n".join((" " * n + line) if line else line for line in _str(s).split("\n"))

    @staticmethod
    def _index(m, *keys):
        for k in keys:
            if m is None:
                return None
            m = m.get(k) if isinstance(m, dict) else m[int(k)]
        return m

    def _include(self, name, dot):
        if name.startswith("templates/") and name[10:] in self.templates:
            return self._render(self.templates[name[10:]], dot, [{"$": self.root}])
        if name not in self.defines:
            raise KeyError(f"template {name!r} not defined")
        return self._render(self.defines[name], dot, [{"$": self.root}])

    # -- expressions
    def _field(self, base, path: List[str]):
        for p in path:
            if p == "":
                continue
            if base is None:
                return None
            if isinstance(base, dict):
                base = base.get(p)
            else:
                base = getattr(base, p, None)
        return base

    def _operand(self, tok: str, dot, scope):
        if tok.startswith('"'):
            return json.loads(tok)
        if tok.startswith("`"):
            return tok[1:-1]
        if re.fullmatch(r"-?\d+", tok):
            return int(tok)
        if re.fullmatch(r"-?\d+\.\d+", tok):
            return float(tok)
        if tok in ("true", "false"):
            return tok == "true"
        if tok == "nil":
            return None
        if tok == ".":
            return dot
        if tok.startswith("."):
            return self._field(dot, tok[1:].split("."))
        if tok.startswith("$"):
            name, _, rest = tok.partition(".")
            for s in reversed(scope):
                if name in s:
                    return self._field(s[name], rest.split(".")) if rest else s[name]
            raise KeyError(f"undefined variable {name}")
        raise ValueError(f"bad operand {tok!r}")

    def _eval(self, toks: List[str], dot, scope):
        """Evaluate a pipeline token list (no declarations)."""
        # split on top-level '|'
        cmds, depth, cur = [], 0, []
        for t in toks:
            if t == "(":
                depth += 1
            elif t == ")":
                depth -= 1
            if t == "|" and depth == 0:
                cmds.append(cur)
                cur = []
            else:
                cur.append(t)
        cmds.append(cur)
        val, have = None, False
        for c in cmds:
            args = self._args(c, dot, scope)
            head = c[0]
            if head in self.funcs:
                fargs = args[1:] + ([val] if have else [])
                val = self.funcs[head](*fargs)
            else:
                if len(args) != 1 or have:
                    raise ValueError(f"cannot call non-function {head!r}")
                val = args[0]
            have = True
        return val

    def _args(self, toks: List[str], dot, scope):
        out, i = [], 0
        while i < len(toks):
            t = toks[i]
            if t == "(":
                depth, j = 1, i + 1
                while depth:
                    depth += {"(": 1, ")": -1}.get(toks[j], 0)
                    j += 1
                out.append(self._eval(toks[i + 1:j - 1], dot, scope))
                i = j
                continue
            if i == 0 and t in self.funcs:
                out.append(t)
            elif t in self.funcs:
                raise ValueError(f"function {t!r} used as an argument; parenthesise it")
            else:
                out.append(self._operand(t, dot, scope))
            i += 1
        return out

    def _pipeline(self, expr: str, dot, scope):
        toks = _tokens(expr)
        if len(toks) >= 2 and toks[1] in (":=", "="):
            v = self._eval(toks[2:], dot, scope)
            if toks[1] == ":=":
                scope[-1][toks[0]] = v
            else:
                for s in reversed(scope):
                    if toks[0] in s:
                        s[toks[0]] = v
                        break
            return None, True
        return self._eval(toks, dot, scope), False

    # -- rendering
    def _render(self, nodes: List[Node], dot, scope) -> str:
        out = []
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Act):
                v, is_decl = self._pipeline(n.expr, dot, scope)
                if not is_decl:
                    out.append(_str(v))
            elif n.kind == "if":
                chosen = None
                if _truthy(self._pipeline(n.expr, dot, scope)[0]):
                    chosen = n.body
                else:
                    for e, body in n.elifs:
                        if _truthy(self._pipeline(e, dot, scope)[0]):
                            chosen = body
                            break
                    else:
                        chosen = n.other
                if chosen:
                    out.append(self._render(chosen, dot, scope + [{}]))
            elif n.kind == "with":
                v = self._pipeline(n.expr, dot, scope)[0]
                if _truthy(v):
                    out.append(self._render(n.body, v, scope + [{}]))
                elif n.other:
                    out.append(self._render(n.other, dot, scope + [{}]))
            elif n.kind == "range":
                expr = n.expr
                names = []
                m = re.match(r"^\s*(\$\w+)(?:\s*,\s*(\$\w+))?\s*:=\s*(.*)$", expr, re.S)
                if m:
                    names = [x for x in (m.group(1), m.group(2)) if x]
                    expr = m.group(3)
                coll = self._pipeline(expr, dot, scope)[0]
                items = list(coll.items()) if isinstance(coll, dict) else \
                    list(enumerate(coll or []))
                if not items and n.other:
                    out.append(self._render(n.other, dot, scope + [{}]))
                for k, v in items:
                    s = {}
                    if len(names) == 1:
                        s[names[0]] = v
                    elif len(names) == 2:
                        s[names[0]], s[names[1]] = k, v
                    out.append(self._render(n.body, v, scope + [s]))
        return "".join(out)

    def render(self) -> Dict[str, str]:
        return {name: self._render(nodes, self.root, [{"$": self.root}])
                for name, nodes in self.templates.items()}

    def manifests(self) -> List[dict]:
        docs = []
        for name, text in self.render().items():
            for d in yaml.safe_load_all(text):
                if d:
                    d.setdefault("_template", name)
                    docs.append(d)
        return docs


# ----------------------------------------------------------------------------- values

def merge(a: dict, b: dict) -> dict:
    out = copy.deepcopy(a)
    for k, v in (b or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _set(values: dict, key: str, raw: str) -> None:
    v: Any = yaml.safe_load(raw) if raw != "" else ""
    parts = key.split(".")
    d = values
    for p in parts[:-1]:
        d = d.setdefault(p, {})
    d[parts[-1]] = v


def chart_values(chart_dir: str, files=(), sets: Optional[Dict[str, str]] = None) -> dict:
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        vals = yaml.safe_load(f) or {}
    for fn in files:
        with open(fn) as f:
            vals = merge(vals, yaml.safe_load(f) or {})
    for k, v in (sets or {}).items():
        _set(vals, k, v)
    return vals


def _sprig_set(d: dict, key: str, value):
    """Sprig `set`: assign in place and return the dict."""
    d[key] = value
    return d


def render_chart(chart_dir: str, files=(), sets=None, release: str = "rel",
                 namespace: str = "default") -> List[dict]:
    return Renderer(chart_dir, chart_values(chart_dir, files, sets), release,
                    namespace).manifests()


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("chart")
    ap.add_argument("-f", "--values", action="append", default=[])
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--release", default="rel")
    a = ap.parse_args(argv)
    sets = dict(s.split("=", 1) for s in a.set)
    print(yaml.safe_dump_all(render_chart(a.chart, a.values, sets, a.release), sort_keys=False))
    return 0


if __name__ == "__main__":
    sys.exit(main())
