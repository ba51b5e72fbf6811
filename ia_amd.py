"""Import shim: exposes the package directory `image-analogies-python_amd/` (a hyphenated name
Python cannot import directly) as the package `ia_amd`.

    import ia_amd
    from ia_amd import config as c
    from ia_amd.image_analogies import image_analogies_main
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'image-analogies-python_amd')
_spec = importlib.util.spec_from_file_location('ia_amd', os.path.join(_DIR, '__init__.py'),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules['ia_amd'] = _mod
_spec.loader.exec_module(_mod)
