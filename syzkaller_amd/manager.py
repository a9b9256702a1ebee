"""Manager-side coverage callers (syz-manager/manager.go) over libsyzcov:

  minimize_corpus   Manager.minimizeCorpus (:504-524): group by call, Minimize
                    per group, rebuild the corpus from the kept inputs;
  CorpusCover       Manager.NewInput's corpusCover merge (:596-621): an input
                    is accepted iff it adds a PC to corpusCover[call], which
                    is then Union-ed with it.  A batch of inputs is checked in
                    one device call (syzcov_newcov_batch with an empty flakes
                    set, which is exactly this predicate and update, applied
                    in batch order);
  summary_stats     httpSummary's per-call coverage table (html.go:67-99);
  corpus_stats      httpCorpus's per-input cover / unique-cover (:157-175).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import cover
from .fuzzer import CoverState


@dataclass
class RpcInput:  # rpctype/rpctype.go:8-13
    Call: str
    Prog: bytes
    CallIndex: int
    Cover: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.uint32))


def minimize_corpus(corpus: list, call_ids: dict | None = None, variant: int = 0) -> list:
    """manager.go:504-524.  `call_ids` maps RpcInput.Call to an integer key
    (sys.CallID in the reference); by default names are numbered in sorted
    order.  Returns the new corpus list."""
    if not corpus:
        return []
    if call_ids is None:
        call_ids = {c: i for i, c in enumerate(sorted({inp.Call for inp in corpus}))}
    calls = [call_ids[inp.Call] for inp in corpus]
    kept = cover.MinimizeCorpus(calls, [inp.Cover for inp in corpus], variant)
    return [corpus[i] for i in kept]


class CorpusCover:
    """mgr.corpusCover: per-CallID union of accepted inputs' covers, resident
    on the device over the PC window [pc_lo, pc_lo + pc_span)."""

    def __init__(self, ncalls: int, pc_lo: int = 0, pc_span: int = 1 << 32):
        self.state = CoverState(ncalls, pc_lo, pc_span)

    def new_inputs(self, call_ids, covers) -> np.ndarray:
        """Accept flags for NewInput calls in arrival order (manager.go:605-610)."""
        return self.state.new_coverage(call_ids, covers).astype(bool)

    def get(self, call: int) -> np.ndarray:
        return self.state.max_cover(call)

    def close(self):
        self.state.close()


@dataclass
class UICallType:  # html.go:427-432
    Name: str
    Inputs: int
    Cover: int
    UniqueCover: int


def summary_stats(corpus: list) -> tuple[list, int]:
    """httpSummary (html.go:67-99): one UICallType per call, sorted by Name
    (UICallTypeArray.Less, :446), and the "cover" stat (len of the union of
    every call's cover).  One device call (syzcov_ui_stats)."""
    names = sorted({inp.Call for inp in corpus})
    gid = {c: i for i, c in enumerate(names)}
    inputs, cov, ucov, _, total = cover.UIStats([inp.Cover for inp in corpus],
                                                [gid[inp.Call] for inp in corpus], len(names))
    return [UICallType(c, int(inputs[i]), int(cov[i]), int(ucov[i])) for i, c in enumerate(names)], total


@dataclass
class UIInput:  # html.go:434-441 (Short/Full need prog.Deserialize: not coverage work)
    N: int
    Cover: int
    UniqueCover: int


def corpus_stats(corpus: list, call: str) -> list:
    """httpCorpus (html.go:157-175): the inputs of `call` with len(Cover) and
    len(Intersection(Cover, uniqueCover(false))), in the order Go's
    sort.Sort(UIInputArray) leaves them (Less = Cover >, :452) -- the same
    comparator as Minimize's sort, so the device restatement of sort.Sort
    gives the reference's tie order too."""
    if not corpus:
        return []
    _, _, _, inu, _ = cover.UIStats([inp.Cover for inp in corpus], [0] * len(corpus), 1)
    data = [UIInput(i, len(inp.Cover), int(inu[i])) for i, inp in enumerate(corpus) if inp.Call == call]
    order = cover.SortOrder([d.Cover for d in data]) if data else []
    return [data[j] for j in order]
