// Link anchors for plugin families not yet split into their own files.
namespace xsched {
void link_noderesources_plugin() {}
void link_trimaran_plugins() {}
void link_sample_plugins() {}
}  // namespace xsched
