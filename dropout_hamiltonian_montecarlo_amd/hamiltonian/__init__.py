"""Mirror of the reference package ``hamiltonian`` (/root/reference/hamiltonian) backed by libhmcx."""
