"""Module registries (reference inference/v2/modules/module_registry.py ``DSModuleRegistryBase``):
one registry per interface (linear, attention, moe, embed, norm); an implementation registers a
name, a ``supports(config)`` predicate and a constructor. heuristics.py asks the registry for the
first implementation, in priority order, that supports the config -- or for a named one when the
user pins it (``RaggedInferenceEngineConfig.implementations``)."""


class ModuleRegistry:
    def __init__(self, interface):
        self.interface = interface
        self._impls = []  # (priority, name, cls)

    def register(self, name, priority=0):
        def deco(cls):
            cls.impl_name = name
            self._impls.append((priority, name, cls))
            self._impls.sort(key=lambda t: -t[0])
            return cls
        return deco

    def names(self):
        return [n for _, n, _ in self._impls]

    def supporting(self, config):
        return [n for _, n, c in self._impls if c.supports(config)]

    def instantiate(self, config, *args, name=None, **kwargs):
        for _, n, cls in self._impls:
            if (name is None or n == name) and cls.supports(config):
                return cls(config, *args, **kwargs)
        if name is not None:
            raise ValueError(f"{self.interface} implementation {name!r} does not exist or does not support {config}")
        raise ValueError(f"no {self.interface} implementation supports {config}")


REGISTRIES = {k: ModuleRegistry(k) for k in ("linear", "attention", "moe", "embed", "norm")}


def register(interface, name, priority=0):
    return REGISTRIES[interface].register(name, priority)
