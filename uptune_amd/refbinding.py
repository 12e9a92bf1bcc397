"""Reference-side binding: the GPU techniques as the reference's own SearchTechniques.

A maintainer drops a four-line module into the reference's technique
directory; `all_techniques()` auto-imports it
(opentuner/search/technique.py:331-338) and it calls `register_all` here.

Each GPU technique is wrapped in a subclass of the REFERENCE's
`SearchTechnique` (technique.py:70-175) that delegates to an inner
uptune_amd technique:

  * desired_result() is the reference's own (technique.py:88-111): it turns
    the dict desired_configuration() returns into a Configuration with
    driver.get_configuration(), builds the ORM DesiredResult and registers
    handle_requested_result -- so the reference driver gets its own row types;
  * desired_configuration() / handle_requested_result() go to the inner GPU
    technique, which reads the driver only through the reference
    SearchDriver/DriverBase surface (requests_query() for the dedup set,
    results_query() for the GP training set, best_result, objective.lt,
    result.configuration.data / .hash; technique.SharedModel);
  * composition rather than multiple inheritance: the reference's
    SearchTechniqueBase.__init__ takes only `name`, so the GPU technique's
    own arguments stay on the inner object.

Instances are deep-copied into every SearchDriver (driver.py:75); the inner
technique's __deepcopy__ drops device state, which is re-created lazily.
"""
from __future__ import annotations

from typing import Any, List, Optional

from . import technique as gpu


def wrap_class(gpu_cls, SearchTechnique):
    """-> a subclass of the reference's SearchTechnique running `gpu_cls`"""

    class Ref(SearchTechnique):
        gpu_class = gpu_cls

        def __init__(self, name: Optional[str] = None, **kw):
            self.gpu = gpu_cls(name=name, **kw)
            super().__init__(name=self.gpu.name)

        def set_driver(self, driver):
            super().set_driver(driver)          # reference: driver, manipulator, objective, add_plugin
            self.gpu.set_driver(driver)

        def desired_configuration(self):
            return self.gpu.desired_configuration()

        def handle_requested_result(self, result):
            self.gpu.handle_requested_result(result)

        def is_ready(self):
            return self.gpu.is_ready()

    Ref.__name__ = Ref.__qualname__ = gpu_cls.__name__
    return Ref


def reference_techniques(SearchTechnique, bandit_cls=None, **kw) -> List[Any]:
    """the GPU counterparts of the reference's population techniques
    (technique.reference_registry), wrapped for the reference driver"""
    return gpu.reference_registry(wrap=lambda c: wrap_class(c, SearchTechnique), bandit_cls=bandit_cls, **kw)


def register_all(technique_module, bandit_cls=None, **kw) -> List[Any]:
    """register every wrapped GPU technique with the reference
    (technique.register, technique.py:287-288); returns them"""
    ts = reference_techniques(technique_module.SearchTechnique, bandit_cls=bandit_cls, **kw)
    for t in ts:
        technique_module.register(t)
    return ts
