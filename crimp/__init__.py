"""``crimp`` import name for the MI355X build: ``from crimp.periodsearch import PeriodSearch`` and every other
``crimp.<module>`` of the photon hot path resolve to the drop-in module ``crimp_amd.<module>`` (the same module
object, so state and classes are shared). Modules the build does not provide (plotting, timing-model fitting,
SURVEY.md section 2 out of scope) raise ImportError as a missing module would."""
import importlib
import importlib.abc
import importlib.util
import sys

from crimp_amd import __version__  # noqa: F401


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if not fullname.startswith("crimp.") or fullname.count(".") != 1:
            return None
        if importlib.util.find_spec("crimp_amd." + fullname.split(".", 1)[1]) is None:
            return None
        return importlib.util.spec_from_loader(fullname, self)

    def create_module(self, spec):
        return importlib.import_module("crimp_amd." + spec.name.split(".", 1)[1])

    def exec_module(self, module):
        pass


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())
