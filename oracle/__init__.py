"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/binding.py).  Never imported by the product."""
