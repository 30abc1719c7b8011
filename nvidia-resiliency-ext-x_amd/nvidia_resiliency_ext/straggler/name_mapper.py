"""Dense integer ids for kernel / section names, identical on every rank.

Reference: straggler/name_mapper.py:22-161.  Ids are consecutive from 0, never change once
assigned, and are assigned in gathered order: all ranks' section names first, then all
ranks' kernel names, rank by rank in list order.  Names are exchanged (all_gather_object)
only when some rank holds a name without an id (one MIN all-reduce of a flag otherwise).
"""
import itertools
from typing import Dict, List

from .dist_utils import all_gather_object, is_all_true


class NameMapper:
    def __init__(self, pg=None):
        self.group = pg
        self.kernel_name_to_id: Dict[str, int] = {}
        self.id_to_kernel_name: Dict[int, str] = {}
        self.section_name_to_id: Dict[str, int] = {}
        self.id_to_section_name: Dict[int, str] = {}
        self.kernel_counter: int = 0
        self.section_counter: int = 0

    def _check_if_has_all_names(self, kernel_names: List[str], section_names: List[str]) -> bool:
        k = self.kernel_name_to_id
        s = self.section_name_to_id
        return all(n in k for n in kernel_names) and all(n in s for n in section_names)

    def gather_and_assign_ids(self, kernel_names: List[str], section_names: List[str],
                              kernels_known: bool = False) -> None:
        """kernels_known: the caller knows every kernel name already has an id (the same names as
        its previous call), so only the sections are looked up; the collective is unchanged."""
        have = (all(n in self.section_name_to_id for n in section_names) if kernels_known else
                self._check_if_has_all_names(kernel_names, section_names))
        if is_all_true(have, self.group):
            return
        gathered = all_gather_object((section_names, kernel_names), self.group)
        for name in itertools.chain.from_iterable(s for s, _ in gathered):
            self._assign_section_id(name)
        for name in itertools.chain.from_iterable(k for _, k in gathered):
            self._assign_kernel_id(name)

    def _assign_kernel_id(self, kernel_name: str) -> int:
        if kernel_name not in self.kernel_name_to_id:
            self.kernel_name_to_id[kernel_name] = self.kernel_counter
            self.id_to_kernel_name[self.kernel_counter] = kernel_name
            self.kernel_counter += 1
        return self.kernel_name_to_id[kernel_name]

    def _assign_section_id(self, section_name: str) -> int:
        if section_name not in self.section_name_to_id:
            self.section_name_to_id[section_name] = self.section_counter
            self.id_to_section_name[self.section_counter] = section_name
            self.section_counter += 1
        return self.section_name_to_id[section_name]

    def get_kernel_name(self, kernel_id: int) -> str:
        return self.id_to_kernel_name[kernel_id]

    def get_kernel_id(self, kernel_name: str) -> int:
        return self.kernel_name_to_id[kernel_name]

    def get_section_name(self, section_id: int) -> str:
        return self.id_to_section_name[section_id]

    def get_section_id(self, section_name: str) -> int:
        return self.section_name_to_id[section_name]
