"""Render the Helm chart without helm: the Go text/template subset charts/mivgpu uses.

There is no helm binary (and no network) in the build environment, so the
chart tests render it here -- ``if / else if / else``, ``with``, ``range``,
``define`` / ``include`` / ``template``, variables, pipelines and the Sprig
functions the templates call (default, printf, print, quote, nindent, indent,
toYaml, toJson, trimSuffix, trunc, sha256sum, dict, list, not, and, or, eq,
ne, empty, required, regexReplaceAll) -- and parse every document with a YAML parser, the way
``helm template | kubeconform`` would in CI.  The reference's chart is checked
the same way by its CI (``hack/verify-chart-version.sh`` + helm lint).

    python hack/helmlite.py charts/mivgpu [--set a.b=c ...]   # prints the manifests
"""

from __future__ import annotations

import hashlib
import json
import re
import sys
from pathlib import Path

import yaml

_ACTION = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------- lexing
def _lex(src: str):
    """-> list of ("text", s) / ("act", s) with Go's {{- -}} trimming applied."""
    out, pos = [], 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip(" \t\r\n")
        if out and out[-1][0] == "trim":
            out.pop()
            text = text.lstrip(" \t\r\n")
        out.append(("text", text))
        body = m.group(2)
        if not body.startswith("/*"):
            out.append(("act", body))
        if m.group(3):
            out.append(("trim", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "trim":
        out.pop()
        text = text.lstrip(" \t\r\n")
    out.append(("text", text))
    return [t for t in out if t[0] != "trim"]


_TOKEN = re.compile(r'\s*(?:(?P<str>"(?:[^"\\]|\\.)*"|`[^`]*`)|(?P<num>-?\d+(?:\.\d+)?)|(?P<op>:=|=|\||\(|\))'
                    r'|(?P<word>[$.A-Za-z_][\w.$]*))')


def _tokens(s: str):
    out, pos = [], 0
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise TemplateError(f"cannot tokenize {s[pos:]!r}")
        for k in ("str", "num", "op", "word"):
            if m.group(k) is not None:
                out.append((k, m.group(k)))
                break
        pos = m.end()
    return out


# ------------------------------------------------------------------ parsing
def _parse_pipeline(toks: list, i: int = 0, stop=(")",)):
    """-> ([cmd, ...], i) where cmd = [operand, ...]"""
    cmds, cur = [], []
    while i < len(toks):
        k, v = toks[i]
        if k == "op" and v in stop:
            break
        if k == "op" and v == "|":
            cmds.append(cur)
            cur = []
            i += 1
            continue
        if k == "op" and v == "(":
            sub, i = _parse_pipeline(toks, i + 1)
            if i >= len(toks) or toks[i] != ("op", ")"):
                raise TemplateError("unbalanced (")
            cur.append(("pipe", sub))
            i += 1
            continue
        if k == "str":
            cur.append(("lit", json.loads(v) if v.startswith('"') else v[1:-1]))
        elif k == "num":
            cur.append(("lit", float(v) if "." in v else int(v)))
        elif v in ("true", "false"):
            cur.append(("lit", v == "true"))
        elif v == "nil":
            cur.append(("lit", None))
        elif v.startswith(".") or v.startswith("$"):
            cur.append(("ref", v))
        else:
            cur.append(("fn", v))
        i += 1
    cmds.append(cur)
    return cmds, i


class Node:
    def __init__(self, kind, **kw):
        self.kind = kind
        self.__dict__.update(kw)


def _parse(tokens, defines: dict):
    """-> list of nodes; fills ``defines``."""
    pos = 0

    def block(terms):
        nonlocal pos
        body = []
        while pos < len(tokens):
            kind, s = tokens[pos]
            if kind == "text":
                body.append(Node("text", s=s))
                pos += 1
                continue
            word = s.split(None, 1)[0] if s else ""
            rest = s[len(word):].strip()
            if word in terms or (word == "else" and "else" in terms):
                return body, word, rest
            pos += 1
            if word in ("if", "with", "range"):
                then, t, r = block(("else", "end"))
                branches = [(rest, then)]
                els = None
                while t == "else":
                    pos += 1
                    if r.startswith("if "):
                        b, t, r2 = block(("else", "end"))
                        branches.append((r[3:].strip(), b))
                        r = r2
                    else:
                        els, t, r = block(("end",))
                pos += 1   # end
                body.append(Node(word, branches=branches, els=els))
            elif word == "define":
                name = json.loads(rest)
                b, _, _ = block(("end",))
                pos += 1
                defines[name] = b
            elif word in ("end", "else"):
                raise TemplateError(f"unexpected {word}")
            else:
                body.append(Node("act", s=s))
        if terms:
            raise TemplateError(f"missing {terms}")
        return body, None, None

    nodes, _, _ = block(())
    return nodes


# ---------------------------------------------------------------- runtime
def _truthy(v) -> bool:
    return not (v is None or v is False or v == 0 or v == "" or (isinstance(v, (list, dict, tuple)) and not v))


def _to_str(v) -> str:
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


def _printf(fmt: str, *args):
    out, ai = [], 0
    i = 0
    while i < len(fmt):
        c = fmt[i]
        if c == "%" and i + 1 < len(fmt):
            f = fmt[i + 1]
            i += 2
            if f == "%":
                out.append("%")
                continue
            a = args[ai] if ai < len(args) else None
            ai += 1
            out.append(_to_str(a) if f in "sv" else (str(int(a)) if f == "d" else json.dumps(a) if f == "q" else
                                                        _to_str(a)))
            continue
        out.append(c)
        i += 1
    return "".join(out)


def _to_yaml(v) -> str:
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=False).rstrip("\n")


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + line if line else line for line in _to_str(s).split("\n"))


class Renderer:
    def __init__(self, chart_dir: Path, values: dict, release: str = "mivgpu", namespace: str = "kube-system",
                 kube_version=("1", "29")):
        self.chart_dir = Path(chart_dir)
        self.chart = yaml.safe_load((self.chart_dir / "Chart.yaml").read_text())
        self.values = values
        self.defines: dict = {}
        self.files: dict = {}
        base = f"{self.chart['name']}/templates"
        for f in sorted((self.chart_dir / "templates").rglob("*")):
            if f.is_dir():
                continue
            rel = f"{base}/{f.relative_to(self.chart_dir / 'templates')}"
            nodes = _parse(_lex(f.read_text()), self.defines)
            self.files[rel] = nodes
            self.defines[rel] = nodes
        self.root = {"Values": values, "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
                     "Chart": {"Name": self.chart["name"], "Version": self.chart["version"],
                               "AppVersion": self.chart.get("appVersion", "")},
                     "Capabilities": {"KubeVersion": {"Major": kube_version[0], "Minor": kube_version[1],
                                                      "Version": f"v{kube_version[0]}.{kube_version[1]}.0"}},
                     "Template": {"BasePath": base}}
        self.funcs = {
            "include": lambda name, ctx: self._run(self.defines[name], ctx, {"$": self.root}),
            "print": lambda *a: "".join(_to_str(x) for x in a),
            "printf": _printf, "quote": lambda *a: " ".join(json.dumps(_to_str(x)) for x in a),
            "default": lambda d, v=None: v if _truthy(v) else d,
            "nindent": lambda n, s: "\n" + _indent(n, s), "indent": _indent,
            "toYaml": _to_yaml, "toJson": lambda v: json.dumps(v, separators=(",", ":")),
            "trimSuffix": lambda suf, s: s[:-len(suf)] if suf and s.endswith(suf) else s,
            "trunc": lambda n, s: s[:int(n)], "sha256sum": lambda s: hashlib.sha256(s.encode()).hexdigest(),
            "dict": lambda *a: {a[i]: a[i + 1] for i in range(0, len(a) - 1, 2)}, "list": lambda *a: list(a),
            "not": lambda v: not _truthy(v), "eq": lambda a, *b: any(a == x for x in b), "ne": lambda a, b: a != b,
            "empty": lambda v: not _truthy(v), "upper": lambda s: s.upper(), "lower": lambda s: s.lower(),
            "required": self._required, "toString": _to_str,
            "regexReplaceAll": lambda rx, s, repl: re.sub(rx, repl.replace("$", "\\"), _to_str(s)),
        }

    @staticmethod
    def _required(msg, v):
        if not _truthy(v):
            raise TemplateError(msg)
        return v

    # -------------------------------------------------------------- eval
    def _ref(self, ref: str, dot, scope):
        if ref == ".":
            return dot
        if ref.startswith("$"):
            name, _, path = ref.partition(".")
            cur = scope["$"] if name == "$" else scope[name]
        else:
            cur, path = dot, ref[1:]
        for part in [p for p in path.split(".") if p]:
            cur = cur.get(part) if isinstance(cur, dict) else None
        return cur

    def _operand(self, op, dot, scope):
        kind, v = op
        if kind == "lit":
            return v
        if kind == "ref":
            return self._ref(v, dot, scope)
        if kind == "pipe":
            return self._pipeline(v, dot, scope)
        return self._call(v, [], dot, scope)

    def _call(self, name, args, dot, scope):
        if name in ("and", "or"):
            res = None
            for a in args:
                res = a
                if (name == "and") != _truthy(a):
                    return a
            return res
        fn = self.funcs.get(name)
        if fn is None:
            raise TemplateError(f"unknown function {name}")
        return fn(*args)

    def _pipeline(self, cmds, dot, scope, piped=None, has_piped=False):
        val, have = piped, has_piped
        for cmd in cmds:
            if not cmd:
                raise TemplateError("empty command")
            head = cmd[0]
            if head[0] == "fn":
                args = [self._operand(o, dot, scope) for o in cmd[1:]]
                if have:
                    args.append(val)
                val = self._call(head[1], args, dot, scope)
            else:
                if len(cmd) > 1:
                    raise TemplateError(f"cannot call a non-function {head}")
                val = self._operand(head, dot, scope)
            have = True
        return val

    def _expr(self, s: str, dot, scope):
        toks = _tokens(s)
        if len(toks) >= 2 and toks[0][0] == "word" and toks[0][1].startswith("$") and toks[1] in (("op", ":="),
                                                                                                 ("op", "=")):
            cmds, _ = _parse_pipeline(toks, 2)
            scope[toks[0][1]] = self._pipeline(cmds, dot, scope)
            return None, True
        if toks and toks[0] == ("word", "template"):
            cmds, _ = _parse_pipeline(toks, 1)
            name = self._operand(cmds[0][0], dot, scope)
            ctx = self._operand(cmds[0][1], dot, scope) if len(cmds[0]) > 1 else None
            return self._run(self.defines[name], ctx, {"$": self.root}), False
        cmds, i = _parse_pipeline(toks)
        if i != len(toks):
            raise TemplateError(f"trailing tokens in {s!r}")
        return self._pipeline(cmds, dot, scope), False

    def _run(self, nodes, dot, scope) -> str:
        out = []
        for n in nodes:
            if n.kind == "text":
                out.append(n.s)
            elif n.kind == "act":
                v, assign = self._expr(n.s, dot, scope)
                if not assign:
                    out.append(_to_str(v))
            elif n.kind == "if":
                for cond, body in n.branches:
                    if _truthy(self._expr(cond, dot, scope)[0]):
                        out.append(self._run(body, dot, dict(scope)))
                        break
                else:
                    if n.els is not None:
                        out.append(self._run(n.els, dot, dict(scope)))
            elif n.kind == "with":
                v = self._expr(n.branches[0][0], dot, scope)[0]
                if _truthy(v):
                    out.append(self._run(n.branches[0][1], v, dict(scope)))
                elif n.els is not None:
                    out.append(self._run(n.els, dot, dict(scope)))
            elif n.kind == "range":
                spec = n.branches[0][0]
                m = re.match(r"^(\$\w+)\s*(?:,\s*(\$\w+))?\s*:=\s*(.*)$", spec)
                seq = self._expr(m.group(3) if m else spec, dot, scope)[0]
                items = list(seq.items()) if isinstance(seq, dict) else list(enumerate(seq or []))
                if not items and n.els is not None:
                    out.append(self._run(n.els, dot, dict(scope)))
                for k, v in items:
                    sc = dict(scope)
                    if m and m.group(2):
                        sc[m.group(1)], sc[m.group(2)] = k, v
                    elif m:
                        sc[m.group(1)] = v
                    out.append(self._run(n.branches[0][1], v, sc))
        return "".join(out)

    def render(self) -> dict:
        """-> {template path: rendered text} for every non-partial template."""
        out = {}
        for rel, nodes in self.files.items():
            name = rel.rsplit("/", 1)[-1]
            if name.startswith("_") or not name.endswith((".yaml", ".yml")):
                continue
            out[rel] = self._run(nodes, self.root, {"$": self.root})
        return out

    def manifests(self) -> list:
        docs = []
        for rel, text in self.render().items():
            for d in yaml.safe_load_all(text):
                if d:
                    d.setdefault("__source__", rel)
                    docs.append(d)
        return docs


def set_value(values: dict, dotted: str, value):
    cur = values
    parts = dotted.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = value


def load(chart_dir, overrides: dict | None = None, **kw) -> Renderer:
    values = yaml.safe_load((Path(chart_dir) / "values.yaml").read_text()) or {}
    for k, v in (overrides or {}).items():
        set_value(values, k, v)
    return Renderer(Path(chart_dir), values, **kw)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("chart")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args(argv)
    ov = {}
    for kv in a.set:
        k, _, v = kv.partition("=")
        ov[k] = yaml.safe_load(v)
    for rel, text in load(a.chart, ov).render().items():
        if text.strip():
            print(f"---\n# Source: {rel}\n{text.strip()}")


if __name__ == "__main__":
    sys.exit(main())
