"""Go `flag`-package compatible command-line parsing.

The reference CLI is Go's `flag` (reference main.go:29-60, flag.Parse at
main.go:159): flags may be written -name value, -name=value, --name value or
--name=value; booleans are set by a bare -b or -b=false (never "-b false");
parsing stops at the first non-flag argument or "--"; an unknown flag prints
"flag provided but not defined: -x" plus usage and exits 2; -h/-help prints
usage and exits 0.  Same contract as csrc/tools/goflags.h (native tools).
"""
from __future__ import annotations

import sys
from dataclasses import dataclass, field
from typing import Any, Callable


class FlagError(Exception):
    pass


@dataclass
class _Flag:
    name: str
    kind: str  # string | int | float | bool | duration
    default: Any
    usage: str
    value: Any = None
    set_explicitly: bool = False


_DURATION_UNITS = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(s: str) -> float:
    """Go time.ParseDuration subset -> seconds ("30s", "1m30s", "250ms", "0")."""
    s = s.strip()
    if s in ("0", ""):
        return 0.0
    total, i, neg = 0.0, 0, False
    if s[0] in "+-":
        neg = s[0] == "-"
        i = 1
    if i >= len(s):
        raise FlagError(f"time: invalid duration {s!r}")
    while i < len(s):
        j = i
        while j < len(s) and (s[j].isdigit() or s[j] == "."):
            j += 1
        if j == i:
            raise FlagError(f"time: invalid duration {s!r}")
        num = float(s[i:j])
        k = j
        while k < len(s) and not (s[k].isdigit() or s[k] == "."):
            k += 1
        unit = s[j:k]
        if unit not in _DURATION_UNITS:
            raise FlagError(f"time: unknown unit {unit!r} in duration {s!r}")
        total += num * _DURATION_UNITS[unit]
        i = k
    return -total if neg else total


def _parse_int(v: str) -> int:
    v = v.strip()
    neg = v.startswith("-")
    body = v[1:] if neg or v.startswith("+") else v
    if body.lower().startswith("0x"):
        x = int(body, 16)
    elif body.startswith("0") and len(body) > 1 and body.isdigit():
        x = int(body, 8)
    else:
        x = int(body, 10)
    return -x if neg else x


def _parse_bool(v: str) -> bool:
    if v in ("1", "t", "T", "true", "TRUE", "True"):
        return True
    if v in ("0", "f", "F", "false", "FALSE", "False"):
        return False
    raise ValueError(v)


class FlagSet:
    def __init__(self, prog: str):
        self.prog = prog
        self._flags: dict[str, _Flag] = {}
        self.args: list[str] = []

    def _add(self, name, kind, default, usage):
        if name in self._flags:
            raise FlagError(f"flag redefined: {name}")
        self._flags[name] = _Flag(name, kind, default, usage, default)

    def string(self, name: str, default: str, usage: str):
        self._add(name, "string", default, usage)

    def int(self, name: str, default: int, usage: str):
        self._add(name, "int", default, usage)

    def float(self, name: str, default: float, usage: str):
        self._add(name, "float", default, usage)

    def bool(self, name: str, default: bool, usage: str):
        self._add(name, "bool", default, usage)

    def duration(self, name: str, default: float, usage: str):
        self._add(name, "duration", default, usage)

    def __getattr__(self, item: str):
        flags = self.__dict__.get("_flags", {})
        key = item.replace("_", "-")
        if key in flags:
            return flags[key].value
        if item in flags:
            return flags[item].value
        raise AttributeError(item)

    def get(self, name: str):
        return self._flags[name].value

    def was_set(self, name: str) -> bool:
        return self._flags[name].set_explicitly

    def usage(self, out=None) -> str:
        lines = [f"Usage of {self.prog}:"]
        for name in sorted(self._flags):
            f = self._flags[name]
            typ = "" if f.kind == "bool" else f" {f.kind}"
            lines.append(f"  -{name}{typ}")
            d = f.default
            dflt = ""
            if f.kind == "string" and d != "":
                dflt = f' (default "{d}")'
            elif f.kind == "bool" and d:
                dflt = " (default true)"
            elif f.kind in ("int", "float") and d != 0:
                dflt = f" (default {d})"
            elif f.kind == "duration" and d:
                dflt = f" (default {d:g}s)"
            lines.append(f"    \t{f.usage}{dflt}")
        text = "\n".join(lines) + "\n"
        (out or sys.stderr).write(text)
        return text

    def _set(self, f: _Flag, raw: str):
        try:
            if f.kind == "string":
                f.value = raw
            elif f.kind == "int":
                f.value = _parse_int(raw)
            elif f.kind == "float":
                f.value = float(raw)
            elif f.kind == "bool":
                f.value = _parse_bool(raw)
            elif f.kind == "duration":
                f.value = parse_duration(raw)
        except (ValueError, FlagError):
            raise FlagError(f'invalid value "{raw}" for flag -{f.name}: parse error')
        f.set_explicitly = True

    def parse(self, argv: list[str], exit_on_error: bool = True) -> "FlagSet":
        try:
            self._parse(argv)
        except SystemExit:
            raise
        except FlagError as e:
            if not exit_on_error:
                raise
            sys.stderr.write(f"{e}\n")
            self.usage()
            sys.exit(2)
        return self

    def _parse(self, argv: list[str]):
        i = 0
        while i < len(argv):
            a = argv[i]
            if len(a) < 2 or a[0] != "-":
                break
            if a == "--":
                i += 1
                break
            body = a[2:] if a.startswith("--") else a[1:]
            if not body or body[0] in "-=":
                raise FlagError(f"bad flag syntax: {a}")
            name, has_value, value = body, False, ""
            if "=" in body:
                name, value = body.split("=", 1)
                has_value = True
            if name in ("h", "help") and name not in self._flags:
                self.usage()
                sys.exit(0)
            f = self._flags.get(name)
            if f is None:
                raise FlagError(f"flag provided but not defined: -{name}")
            if f.kind == "bool":
                self._set(f, value if has_value else "true")
            else:
                if not has_value:
                    i += 1
                    if i >= len(argv):
                        raise FlagError(f"flag needs an argument: -{name}")
                    value = argv[i]
                self._set(f, value)
            i += 1
        self.args = argv[i:]
