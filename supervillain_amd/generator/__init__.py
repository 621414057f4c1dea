"""Generators: the plugin protocol (generator.py), composition (combining.py) and the MI355X
hot-path generators NeighborhoodUpdate (villain.py), CoexactUpdate and PlaquetteUpdate (worldline.py)."""
from supervillain_amd.generator.generator import Generator
from supervillain_amd.generator import combining, villain, worldline
from supervillain_amd.generator.combining import KeepEvery, Sequentially
