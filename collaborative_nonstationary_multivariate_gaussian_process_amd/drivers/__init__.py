"""Driver entry points of the reference (``code/NMGP_PM25.py``, ``code/NMGP_HCP.py``): ``VTVLCM``.

The reference drivers load ``../data/{PM25,HCP}/*.pickle`` and create result directories at import
time (``NMGP_PM25.py:17-38``, ``NMGP_HCP.py:14-37``); those data are not shipped with the reference
(``ReadMe.txt:7``).  Here the data are injected (``set_data``), read from a file the user names
(``load_data``) or generated (``synthetic_data``), and ``VTVLCM`` keeps the reference's signature and
return values, calling this package's ``inference`` with the same keyword arguments.
"""
from . import NMGP_HCP, NMGP_PM25  # noqa: F401
from ._common import synthetic_data  # noqa: F401
