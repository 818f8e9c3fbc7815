// Force-links every plugin translation unit so their static registrars run
// even when the core is linked from an archive.
#include "framework/plugin.h"

namespace xsched {

void link_intree_plugins();
void link_flexgpu_plugin();
void link_coscheduling_plugin();
void link_preemption_plugins();
void link_capacity_plugin();
void link_noderesources_plugin();
void link_nrt_plugin();
void link_trimaran_plugins();
void link_sample_plugins();
void link_topology_plugins();
void link_crossnode_plugin();
void link_volume_plugins();

void register_builtin_plugins() {
  link_intree_plugins();
  link_flexgpu_plugin();
  link_coscheduling_plugin();
  link_preemption_plugins();
  link_capacity_plugin();
  link_noderesources_plugin();
  link_nrt_plugin();
  link_trimaran_plugins();
  link_sample_plugins();
  link_topology_plugins();
  link_crossnode_plugin();
  link_volume_plugins();
}

}  // namespace xsched
