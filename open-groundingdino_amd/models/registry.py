"""Build-function registry (reference models/registry.py:12-57).  main.py looks
the model up with ``MODULE_BUILD_FUNCS.get(args.modelname)``."""
import inspect
from functools import partial


class Registry:
    def __init__(self, name):
        self._name = name
        self._module_dict = {}

    def __repr__(self):
        return f"{self.__class__.__name__}(name={self._name}, items={list(self._module_dict)})"

    def __len__(self):
        return len(self._module_dict)

    @property
    def name(self):
        return self._name

    @property
    def module_dict(self):
        return self._module_dict

    def get(self, key):
        return self._module_dict.get(key)

    def registe_with_name(self, module_name=None, force=False):
        return partial(self.register, module_name=module_name, force=force)

    def register(self, module_build_function, module_name=None, force=False):
        if not inspect.isfunction(module_build_function):
            raise TypeError(f"module_build_function must be a function, but got {type(module_build_function)}")
        name = module_name or module_build_function.__name__
        if not force and name in self._module_dict:
            raise KeyError(f"{name} is already registered in {self._name}")
        self._module_dict[name] = module_build_function
        return module_build_function


MODULE_BUILD_FUNCS = Registry("model build functions")
