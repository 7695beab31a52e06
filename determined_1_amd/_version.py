__version__ = "0.13.10.dev0+mi355x"
