"""Minimal config loader replacing mmcv.Config (absent): executes a plain-Python
config file (the reference's configs/*.py format) and wraps its dicts in
attribute-access ConfigDicts, which is all the reference's code needs
(`train_cfg.rpn.assigner`, `'sampler' in cfg`, `cfg.get(...)`)."""
import runpy


class ConfigDict(dict):
    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = value


def wrap(obj):
    if isinstance(obj, dict) and not isinstance(obj, ConfigDict):
        return ConfigDict({k: wrap(v) for k, v in obj.items()})
    if isinstance(obj, list):
        return [wrap(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(wrap(v) for v in obj)
    return obj


class Config(ConfigDict):
    @staticmethod
    def fromfile(path):
        ns = runpy.run_path(path)
        return Config({k: wrap(v) for k, v in ns.items() if not k.startswith('__')})
