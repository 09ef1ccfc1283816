"""Hydra-compatible configuration composer on PyYAML (Hydra / omegaconf are not available).

Reference usage: ``@hydra.main(config_path="conf", config_name=...)`` in main.py:134, eval.py:193,
save_features.py:119, supervised.py:165 with Hydra 1.0 semantics:

* defaults list with config groups (``- experiment: cifar10``, ``- hydra/output: custom``),
  ``_self_`` supported (absent ⇒ Hydra 1.0 order: primary config first, then defaults);
* ``# @package _global_`` / ``_group_`` headers (group files default to ``_global_``);
* CLI overrides: ``group=option`` (group selection), ``a.b=value`` (must exist — struct mode),
  ``+a.b=value`` (add), ``++a.b=value`` (add or override), ``~a.b`` (delete); values parsed like
  YAML (ints, floats incl. ``1e-4``, bools, null, lists) else strings;
* interpolation ``${a.b}``, ``${now:%Y-%m-%d}``, ``${env:VAR}``/``${oc.env:VAR,default}``,
  ``${hydra.job.num}`` / ``${hydra.job.name}``;
* ``-m/--multirun`` sweeps over comma-separated values (cartesian product, sequential jobs,
  ``hydra.sweep.dir``/``subdir``);
* run directory creation + chdir + ``.hydra/{config,hydra,overrides}.yaml`` + job log file
  (``<job>.log``) exactly where Hydra would put them.

The reference's YAML files load unchanged (``conf/`` here keeps their keys and defaults and only
adds optional keys).
"""
from __future__ import annotations

import copy
import datetime
import functools
import itertools
import logging
import os
import re
import sys
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import yaml


# ----------------------------------------------------------------------------- YAML loading
class _Loader(yaml.SafeLoader):
    pass


# YAML 1.1 (PyYAML) reads "1e-4" as a string; OmegaConf/Hydra read it as a float.
_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
        |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
        |\.[0-9_]+(?:[eE][-+][0-9]+)?
        |[-+]?\.(?:inf|Inf|INF)
        |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."))


def load_yaml_text(text: str) -> Any:
    return yaml.load(text, Loader=_Loader)


def _read_package(text: str) -> Optional[str]:
    for line in text.splitlines():
        s = line.strip()
        if not s:
            continue
        if not s.startswith("#"):
            break
        m = re.match(r"#\s*@package\s+(\S+)", s)
        if m:
            return m.group(1)
    return None


# ----------------------------------------------------------------------------- config object
class Config(dict):
    """dict with attribute access; nested dicts are Config too (OmegaConf DictConfig subset)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return Config({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def to_dict(self) -> dict:
        return _plain(self)

    def select(self, dotted: str, default=None):
        cur = self
        for part in dotted.split("."):
            if isinstance(cur, dict) and part in cur:
                cur = cur[part]
            else:
                return default
        return cur


def _wrap(obj):
    if isinstance(obj, dict):
        return Config({k: _wrap(v) for k, v in obj.items()})
    if isinstance(obj, list):
        return [_wrap(v) for v in obj]
    return obj


def _plain(obj):
    if isinstance(obj, dict):
        return {k: _plain(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_plain(v) for v in obj]
    return obj


def _merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if k == "defaults":
            continue
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _nest(package: str, node: dict) -> dict:
    if not package:
        return node
    out = node
    for part in reversed(package.split(".")):
        out = {part: out}
    return out


# ----------------------------------------------------------------------------- overrides
class ConfigCompositionError(Exception):
    pass


def parse_value(s: str) -> Any:
    if s == "":
        return ""
    try:
        v = load_yaml_text(s)
    except yaml.YAMLError:
        return s
    if isinstance(v, (dict,)):
        return s
    return v


def _split_sweep(value: str) -> List[str]:
    # split on commas not inside brackets / quotes
    parts, depth, cur, quote = [], 0, "", None
    for ch in value:
        if quote:
            cur += ch
            if ch == quote:
                quote = None
            continue
        if ch in "'\"":
            quote = ch
            cur += ch
        elif ch in "[{(":
            depth += 1
            cur += ch
        elif ch in "]})":
            depth -= 1
            cur += ch
        elif ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    return parts


def _set_dotted(cfg: dict, key: str, value: Any, mode: str) -> None:
    parts = key.split(".")
    cur = cfg
    for i, p in enumerate(parts[:-1]):
        if p not in cur or not isinstance(cur[p], dict):
            if mode == "set":
                raise ConfigCompositionError(
                    f"Could not override '{key}': key '{'.'.join(parts[:i + 1])}' is not in the "
                    f"config. To append to your config use +{key}=...")
            cur[p] = {}
        cur = cur[p]
    last = parts[-1]
    if mode == "set" and last not in cur:
        raise ConfigCompositionError(
            f"Could not override '{key}': key '{key}' is not in the config. "
            f"To append to your config use +{key}=...")
    if mode == "add" and last in cur:
        raise ConfigCompositionError(f"Could not append to config. An item is already at '{key}'")
    cur[last] = value


def _del_dotted(cfg: dict, key: str) -> None:
    parts = key.split(".")
    cur = cfg
    for p in parts[:-1]:
        cur = cur[p]
    cur.pop(parts[-1], None)


# ----------------------------------------------------------------------------- interpolation
_INTERP = re.compile(r"\$\{([^${}]+)\}")


def _resolve_all(cfg: dict, now: datetime.datetime) -> dict:
    root = cfg

    def lookup(expr: str, stack: Tuple[str, ...]):
        expr = expr.strip()
        if expr.startswith("now:"):
            return now.strftime(expr[4:])
        if expr.startswith("env:") or expr.startswith("oc.env:"):
            body = expr.split(":", 1)[1]
            name, _, default = body.partition(",")
            v = os.environ.get(name.strip())
            if v is None:
                if default:
                    return parse_value(default.strip())
                raise ConfigCompositionError(f"environment variable '{name}' not found")
            return v
        if expr in stack:
            raise ConfigCompositionError(f"interpolation cycle at ${{{expr}}}")
        cur: Any = root
        for part in expr.split("."):
            if isinstance(cur, dict) and part in cur:
                cur = cur[part]
            elif isinstance(cur, list) and part.isdigit():
                cur = cur[int(part)]
            else:
                raise ConfigCompositionError(f"interpolation key '{expr}' not found")
        return resolve(cur, stack + (expr,))

    def resolve(v, stack=()):
        if isinstance(v, str) and "${" in v:
            m = _INTERP.fullmatch(v)
            if m:
                return lookup(m.group(1), stack)
            return _INTERP.sub(lambda mm: str(lookup(mm.group(1), stack)), v)
        if isinstance(v, dict):
            return {k: resolve(x, stack) for k, x in v.items()}
        if isinstance(v, list):
            return [resolve(x, stack) for x in v]
        return v

    # resolve repeatedly until fixed point (values referencing other interpolated values)
    out = cfg
    for _ in range(8):
        new = resolve(out)
        root = new
        if new == out:
            break
        out = new
    return out


# ----------------------------------------------------------------------------- composition
class Composer:
    def __init__(self, config_dir: str):
        self.dir = Path(config_dir)

    def _load(self, rel: str) -> Tuple[dict, Optional[str]]:
        p = self.dir / (rel + ".yaml")
        if not p.exists():
            raise ConfigCompositionError(f"Could not load {rel} (looked for {p})")
        text = p.read_text()
        node = load_yaml_text(text) or {}
        return node, _read_package(text)

    def group_options(self, group: str) -> List[str]:
        d = self.dir / group
        return sorted(p.stem for p in d.glob("*.yaml")) if d.is_dir() else []

    def compose(self, config_name: str, overrides: Sequence[str] = ()) -> Config:
        primary, _pkg = self._load(config_name)
        defaults = list(primary.get("defaults", []) or [])
        groups: Dict[str, Optional[str]] = {}
        order: List[str] = []
        has_self = False
        for d in defaults:
            if isinstance(d, dict):
                for g, opt in d.items():
                    groups[g] = opt
                    order.append(g)
            elif d == "_self_":
                has_self = True
                order.append("_self_")
            else:
                order.append("file:" + str(d))
        if not has_self:
            order.insert(0, "_self_")  # Hydra 1.0: primary config, then defaults
        value_ovr: List[Tuple[str, str, Any]] = []
        for o in overrides:
            o = o.strip()
            if not o:
                continue
            if o.startswith("~"):
                value_ovr.append(("del", o[1:].split("=")[0], None))
                continue
            if "=" not in o:
                raise ConfigCompositionError(f"Error parsing override '{o}': missing '='")
            k, v = o.split("=", 1)
            mode = "set"
            if k.startswith("++"):
                mode, k = "force", k[2:]
            elif k.startswith("+"):
                mode, k = "add", k[1:]
            if k in groups or (mode == "add" and (self.dir / k).is_dir()):
                if k not in groups:
                    order.append(k)
                groups[k] = v if v not in ("null", "None") else None
                continue
            value_ovr.append((mode, k, parse_value(v)))
        cfg: dict = {}
        for item in order:
            if item == "_self_":
                _merge(cfg, {k: v for k, v in primary.items() if k != "defaults"})
            elif item.startswith("file:"):
                node, pkg = self._load(item[5:])
                _merge(cfg, node)
            else:
                opt = groups.get(item)
                if opt is None:
                    continue
                node, pkg = self._load(f"{item}/{opt}")
                if pkg is None or pkg == "_global_":
                    _merge(cfg, node)
                elif pkg == "_group_":
                    _merge(cfg, _nest(item.replace("/", "."), node))
                else:
                    _merge(cfg, _nest(pkg, node))
        for mode, k, v in value_ovr:
            if mode == "del":
                _del_dotted(cfg, k)
            else:
                _set_dotted(cfg, k, v, mode)
        return _wrap(cfg)


def compose(config_dir: str, config_name: str, overrides: Sequence[str] = (),
            job_name: str = "app", job_num: int = 0,
            now: Optional[datetime.datetime] = None) -> Config:
    """Compose + resolve (``hydra`` node included, like Hydra's full config)."""
    cfg = Composer(config_dir).compose(config_name, overrides)
    cfg.setdefault("hydra", Config())
    hyd = cfg["hydra"]
    hyd.setdefault("job", Config())
    hyd["job"].setdefault("name", job_name)
    hyd["job"]["num"] = job_num
    hyd["job"]["override_dirname"] = ",".join(sorted(overrides))
    hyd.setdefault("run", Config({"dir": "outputs/${now:%Y-%m-%d}/${now:%H-%M-%S}"}))
    hyd.setdefault("sweep", Config({"dir": "multirun/${now:%Y-%m-%d}/${now:%H-%M-%S}",
                                    "subdir": "${hydra.job.num}"}))
    hyd.setdefault("output_subdir", ".hydra")
    return _wrap(_resolve_all(cfg, now or datetime.datetime.now()))


def task_config(full: Config) -> Config:
    """The config handed to the task function (Hydra strips the ``hydra`` node)."""
    return Config({k: v for k, v in full.items() if k != "hydra"})


def to_yaml(cfg) -> str:
    return yaml.safe_dump(_plain(cfg), sort_keys=False, default_flow_style=False)


# ----------------------------------------------------------------------------- entry decorator
_ORIGINAL_CWD: Optional[str] = None


def get_original_cwd() -> str:
    return _ORIGINAL_CWD or os.getcwd()


def to_absolute_path(path: str) -> str:
    p = Path(path)
    return str(p if p.is_absolute() else Path(get_original_cwd()) / p)


def _setup_logging(run_dir: Path, job_name: str) -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    fmt = logging.Formatter("[%(asctime)s][%(name)s][%(levelname)s] - %(message)s")
    sh = logging.StreamHandler(sys.stdout)
    sh.setFormatter(fmt)
    root.addHandler(sh)
    fh = logging.FileHandler(run_dir / f"{job_name}.log")
    fh.setFormatter(fmt)
    root.addHandler(fh)
    root.setLevel(logging.INFO)


def run_job(task: Callable, config_dir: str, config_name: str, overrides: Sequence[str],
            job_name: str, job_num: int = 0, sweep: bool = False,
            now: Optional[datetime.datetime] = None, chdir: bool = True):
    global _ORIGINAL_CWD
    full = compose(config_dir, config_name, overrides, job_name, job_num, now)
    hyd = full["hydra"]
    run_dir = Path(hyd["sweep"]["dir"]) / str(hyd["sweep"]["subdir"]) if sweep \
        else Path(hyd["run"]["dir"])
    if _ORIGINAL_CWD is None:
        _ORIGINAL_CWD = os.getcwd()
    run_dir = run_dir if run_dir.is_absolute() else Path(_ORIGINAL_CWD) / run_dir
    run_dir.mkdir(parents=True, exist_ok=True)
    sub = run_dir / str(hyd.get("output_subdir", ".hydra"))
    sub.mkdir(parents=True, exist_ok=True)
    task_cfg = task_config(full)
    (sub / "config.yaml").write_text(to_yaml(task_cfg))
    (sub / "hydra.yaml").write_text(to_yaml({"hydra": hyd}))
    (sub / "overrides.yaml").write_text(to_yaml(list(overrides)))
    prev = os.getcwd()
    if chdir:
        os.chdir(run_dir)
    _setup_logging(run_dir, job_name)
    try:
        return task(task_cfg)
    finally:
        if chdir:
            os.chdir(prev)


def hydra_main(config_path: str, config_name: str):
    """Drop-in for ``@hydra.main(config_path=..., config_name=...)`` (argv-driven)."""

    def deco(fn: Callable):
        @functools.wraps(fn)
        def wrapper(argv: Optional[Sequence[str]] = None):
            args = list(sys.argv[1:] if argv is None else argv)
            multirun = False
            if args and args[0] in ("-m", "--multirun"):
                multirun = True
                args = args[1:]
            args = [a for a in args if a not in ("-m", "--multirun")]
            mod = sys.modules.get(fn.__module__)
            base = Path(getattr(mod, "__file__", None) or ".").resolve().parent
            cdir = Path(config_path)
            cdir = cdir if cdir.is_absolute() else base / cdir
            job = Path(getattr(mod, "__file__", "app")).stem if mod else "app"
            now = datetime.datetime.now()
            if not multirun:
                return run_job(fn, str(cdir), config_name, args, job, now=now)
            axes = []
            for a in args:
                k, _, v = a.partition("=")
                vals = _split_sweep(v) if ("," in v and not a.startswith("~")) else [v]
                axes.append([f"{k}={x}" for x in vals])
            results = []
            for num, combo in enumerate(itertools.product(*axes)):
                results.append(run_job(fn, str(cdir), config_name, list(combo), job, num,
                                       sweep=True, now=now))
            return results

        return wrapper

    return deco
