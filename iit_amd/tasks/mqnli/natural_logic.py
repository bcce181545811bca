"""Natural-logic composition tables by model checking (the MQNLI causal model's semantics).

Relations (MacCartney & Manning): ``EQ`` (≡), ``FWD`` (⊏), ``REV`` (⊐), ``NEG`` (^),
``ALT`` (|), ``COV`` (‿), ``IND`` (#).  A relation between two predicates or two
sentences is read off the truth-value combinations that can co-occur: for sets,
each element of a small universe is a "world" ``(u in X, u in Y)``; for sentences,
each model is.  Composition tables (modifier + head, negation projection, and the
generalized-quantifier projection ``Q_p(A_p, B_p)`` vs ``Q_h(A_h, B_h)``) are
computed once by enumerating every configuration of non-degenerate sets over a
4-element universe consistent with the argument relations -- so they are correct
by construction for that model class, rather than transcribed tables.
"""
from __future__ import annotations

import itertools
from functools import lru_cache

import numpy as np

EQ, FWD, REV, NEG, ALT, COV, IND = range(7)
NAMES = ("≡", "⊏", "⊐", "^", "|", "‿", "#")
SOME, EVERY, NO, NOTEVERY = range(4)
QUANTIFIERS = ("some", "every", "no", "not every")
U_SIZE = 4
FULL = (1 << U_SIZE) - 1


def classify(tt: bool, tf: bool, ft: bool, ff: bool) -> int:
    """Relation from which truth combinations (p, h) are possible."""
    p_entails_h, h_entails_p = not tf, not ft
    exclusive, exhaustive = not tt, not ff
    if p_entails_h and h_entails_p:
        return EQ
    if p_entails_h:
        return FWD
    if h_entails_p:
        return REV
    if exclusive and exhaustive:
        return NEG
    if exclusive:
        return ALT
    if exhaustive:
        return COV
    return IND


def set_relation(x: int, y: int) -> int:
    tt = bool(x & y)
    tf = bool(x & ~y & FULL)
    ft = bool(~x & y & FULL)
    ff = bool(~x & ~y & FULL)
    return classify(tt, tf, ft, ff)


@lru_cache(maxsize=None)
def _pairs_by_relation():
    sets = [s for s in range(1, FULL)]  # non-empty, non-universal (general position)
    out = {r: [] for r in range(7)}
    for x in sets:
        for y in sets:
            out[set_relation(x, y)].append((x, y))
    return {r: np.array(v, dtype=np.int64).reshape(-1, 2) for r, v in out.items()}


def _rel_from_pairs(px: np.ndarray, py: np.ndarray) -> int:
    """Relation between the predicate families given all (x, y) realisations."""
    tt = bool(np.any(px & py))
    tf = bool(np.any(px & ~py & FULL))
    ft = bool(np.any(~px & py & FULL))
    ff = bool(np.any(~px & ~py & FULL))
    return classify(tt, tf, ft, ff)


@lru_cache(maxsize=None)
def intersective_table() -> np.ndarray:
    """``T[r_mod, r_head]``: relation of ``M_p ∩ H_p`` vs ``M_h ∩ H_h``."""
    P = _pairs_by_relation()
    T = np.full((7, 7), IND, dtype=np.int64)
    for rm, rh in itertools.product(range(7), range(7)):
        if not len(P[rm]) or not len(P[rh]):
            continue
        m, h = P[rm], P[rh]
        xp = (m[:, None, 0] & h[None, :, 0]).ravel()
        xh = (m[:, None, 1] & h[None, :, 1]).ravel()
        T[rm, rh] = _rel_from_pairs(xp, xh)
    return T


@lru_cache(maxsize=None)
def negation_table() -> np.ndarray:
    """``T[neg_p, neg_h, r]``: relation of ``[not] X_p`` vs ``[not] X_h`` given ``X_p r X_h``."""
    P = _pairs_by_relation()
    T = np.full((2, 2, 7), IND, dtype=np.int64)
    for np_, nh, r in itertools.product(range(2), range(2), range(7)):
        if not len(P[r]):
            continue
        x, y = P[r][:, 0], P[r][:, 1]
        x = (~x & FULL) if np_ else x
        y = (~y & FULL) if nh else y
        T[np_, nh, r] = _rel_from_pairs(x, y)
    return T


def _quantify(q: int, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    if q == SOME:
        return (a & b) != 0
    if q == EVERY:
        return (a & ~b & FULL) == 0
    if q == NO:
        return (a & b) == 0
    return (a & ~b & FULL) != 0  # NOTEVERY


@lru_cache(maxsize=None)
def quantifier_table() -> np.ndarray:
    """``T[q_p, q_h, r_restrictor, r_scope]``: relation of ``Q_p(A_p, B_p)`` vs ``Q_h(A_h, B_h)``."""
    P = _pairs_by_relation()
    T = np.full((4, 4, 7, 7), IND, dtype=np.int64)
    for ra, rb in itertools.product(range(7), range(7)):
        if not len(P[ra]) or not len(P[rb]):
            continue
        A, B = P[ra], P[rb]
        ap, ah = np.repeat(A[:, 0], len(B)), np.repeat(A[:, 1], len(B))
        bp, bh = np.tile(B[:, 0], len(A)), np.tile(B[:, 1], len(A))
        for qp, qh in itertools.product(range(4), range(4)):
            tp, th = _quantify(qp, ap, bp), _quantify(qh, ah, bh)
            T[qp, qh, ra, rb] = classify(bool(np.any(tp & th)), bool(np.any(tp & ~th)), bool(np.any(~tp & th)),
                                         bool(np.any(~tp & ~th)))
    return T


def label_of(rel: int) -> int:
    """3-way NLI label: 0 entailment (≡, ⊏), 1 contradiction (^, |), 2 neutral."""
    return 0 if rel in (EQ, FWD) else (1 if rel in (NEG, ALT) else 2)
