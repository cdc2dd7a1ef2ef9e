"""`python -m ndfl.gunzip InputFile.gz OutputFile` -- S/gunzip.java over the GPU codec (see ndfl.cli)."""
from .cli import _main, gunzip_submain

if __name__ == "__main__":
    _main(gunzip_submain)
