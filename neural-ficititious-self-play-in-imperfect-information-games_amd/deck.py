"""The reference's card deck (leduc/deck.py:5-55, leduc/cardmatrix.py:4-13) for the drop-in.

``install_dropin()`` registers this module as ``leduc.deck`` and its ``Cardmatrix`` as
``leduc.cardmatrix``.  A deck is six cards, ranks 0..2 (0 = Ace, the best) x 2 suits, in
the reference's order; ``shuffle`` consumes the global ``random`` exactly like the
reference's ``random.shuffle`` (``pyrandom``: CPython 3 by default, 2.7 on request), and
``pick_up`` pops from the end.  ``leduc.Env.reset`` deals from this deck on the host and
injects the three ranks into the device env (``nfsp_env_set_deal``); the batched engine
deals on the device from Philox instead (include/nfsp.h).
"""
from __future__ import annotations

from . import pyrandom

RANK_NAMES = ['Ace', 'King', 'Queen', 'Jack', '10', '9', '8', '7', '6', '5', '4', '3', '2']
SUIT_NAMES = ['Heart', 'Spades', 'Cross', 'Diamonds']


class Cardmatrix:
    """leduc/cardmatrix.py:4-13: names of a rank and a suit."""

    def getCard(self, rank, suit):  # noqa: N802 (the reference's name)
        return RANK_NAMES[rank], SUIT_NAMES[suit]


class Card:
    """A card with rank and suit (leduc/deck.py:5-24)."""

    def __init__(self, rank, suit):
        self._rank = rank
        self._suit = suit
        self._named_rank, self._named_suit = Cardmatrix().getCard(rank, suit)

    def __str__(self):
        return f"{self._named_rank} {self._named_suit} {self._rank} {self._suit}"

    @property
    def rank(self):
        return self._rank


class Deck:
    """Six cards, 2 suits x 3 ranks (leduc/deck.py:27-55)."""

    def __init__(self, size=6):
        assert size > 0 and size % 2 == 0, f'deck size must be a positive even number, got {size}'
        self._size = size
        self._fill()
        self.fake_pub = Card(-1, -1)

    def _fill(self):
        self._cards = [Card(rank, suit) for rank in range(self._size // 2) for suit in range(2)]

    def shuffle(self):
        pyrandom.shuffle(self._cards)

    def fake_pub_card(self):
        return self.fake_pub

    def pick_up(self):
        return self._cards.pop()

    def print_deck(self):
        """One line per remaining card, bottom of the deck first (leduc/deck.py:53-55)."""
        if self._cards:
            print("\n".join(map(str, self._cards)))
